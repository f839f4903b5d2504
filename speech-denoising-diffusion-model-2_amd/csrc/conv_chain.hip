// The UNet's bottom level as ONE launch: downs.10 (stride-2 Downsample into the 8x4 image),
// mid.0 (ResnetBlock, identity residual) and ups.0 (ResnetBlock over the skip concat with
// downs.10's output, 1x1 res_conv), UNetModified2.py:103-142, 218-235, 252-265.
//
// At the bottom level an image is 8 x 4 = 32 pixels x 160 channels (10 KB in 16 bits), so one
// block can hold a whole image and every intermediate in LDS; GroupNorm over the image is then a
// block-local reduction, and the five convs run back to back with block barriers instead of five
// dependent launches (each a one-wave grid of 160-256 latency-bound blocks: ~50 us per step,
// DESIGN.md §3a).  Only the level's input (downs.9.block2's output) is read and only ups.0's
// output is written; the four intermediates never reach HBM.
//
// Block = one image, C / 16 waves; wave w owns output channels [16 w, 16 w + 16) of every conv, both
// 16-pixel fragments, and the whole K (taps x 32-channel chunks, then the res_conv chunks), with
// its weight fragments streamed from the MFMA-fragment-major images (ConvArgs::wgt_f layout)
// through a register ring.  Operands: a plane-major zero-bordered image of the GroupNorm+SiLU'd
// input (a plane = 8 channels, 16 B per pixel, 1 KiB plane stride), raw outputs kept compact
// [pixel][C] for the residual, the skip concat and the res_conv.  GroupNorm statistics come from
// the fp32 epilogue values (before the storage rounding, as every conv kernel here), per channel
// over the image, combined per group in a fixed order.
#include "conv_common.h"
#include "kernels.h"

#ifndef SDDM_CHAIN_RING
#define SDDM_CHAIN_RING 20
#endif

namespace sddm {

template <typename T, int C, int H, int W>
struct ChainGeo {
  static constexpr int P = H * W, FP = P / 16, NWV = C / 16, NT = 64 * NWV;
  static constexpr int ES = (int)sizeof(T), VE = 16 / ES;
  static constexpr int HI = 2 * H + 1, WI = 2 * W + 1;                   // downs.10 halo (input rows -1 .. 2H-1)
  static constexpr int PIN = (HI * WI * 16 + 255) / 256 * 256;          // its plane stride
  static constexpr int HP = H + 2, WP = W + 2;                           // stride-1 halo
  static constexpr int PIMG = (HP * WP * 16 + 255) / 256 * 256;          // plane stride
  static constexpr int IN_BYTES = (C / VE) * PIN, IMG_BYTES = (2 * C / VE) * PIMG;
  static constexpr int REG0 = IN_BYTES > IMG_BYTES ? IN_BYTES : IMG_BYTES;   // IN and IMG alias
  static constexpr int RAW = P * C * ES;                                 // one compact raw tensor
  static constexpr int OFF_RD = REG0, OFF_RH = OFF_RD + RAW, OFF_RM = OFF_RH + RAW;
  static constexpr int OFF_ST = OFF_RM + RAW;                            // [4][C][2] mean / var
  static constexpr int OFF_GS = OFF_ST + 4 * C * 2 * 4;                  // [2][2C] scale / shift
  static constexpr int LDS = OFF_GS + 2 * 2 * C * 4;
};

// The weight fragments of a wave's 16 output channels for the five convs form one stream of K
// steps (segments: downs.10, mid.0.block1, mid.0.block2, ups.0.block1, ups.0.block2 3x3, its
// res_conv), read through one D-deep register ring that runs on across the conv boundaries: the
// next conv's first fragments are in flight during this conv's last steps, its GroupNorm and its
// staging.  (A block reads every weight of the level, ~2.9 MB in 16 bits, through one CU: the ring
// depth, i.e. the bytes in flight per wave, sets the level's time.)
template <int C>
struct ChainStream {
  static constexpr int K1 = (C / 32) * 9, K2 = (2 * C / 32) * 9, KR = 2 * C / 32;
  static constexpr int N[6] = {K1, K1, K1, K2, K1, KR};
  static constexpr int S[7] = {0, K1, 2 * K1, 3 * K1, 3 * K1 + K2, 4 * K1 + K2, 4 * K1 + K2 + KR};
};

// stream position q -> this lane's 16-byte piece of that fragment (base[k]: segment k's first
// fragment of this wave, wave-uniform; lane8 = 8 lane); q past the end is clamped
template <typename T, int C>
__device__ __forceinline__ Frag<T> chain_frag(const T* const (&base)[6], int q, int lane8) {
  using SS = ChainStream<C>;
  q = min(q, SS::S[6] - 1);
  int k = 0;
#pragma unroll
  for (int j = 1; j < 6; ++j) k += q >= SS::S[j] ? 1 : 0;
  int st = 0;
#pragma unroll
  for (int j = 1; j < 6; ++j) st = k == j ? SS::S[j] : st;
  const T* b = base[0];
#pragma unroll
  for (int j = 1; j < 6; ++j) b = k == j ? base[j] : b;
  return load_frag<T>((const char*)(b + (size_t)(q - st) * 512 + lane8));
}

// conv SEG of the chain: acc = W (wave wv's 16 output channels) x operand; its 3x3 K steps from `img`
// (plane stride PL, halo row width HW, stride 2 when S2), for SEG 4 then the res_conv steps from
// the raw concat (ra | rb) [P][C] at the output pixels.  Ring slot of stream position q: q % D
// (compile-time: the segment starts are)
template <typename T, int C, int H, int W, int D, int SEG>
__device__ __forceinline__ void chain_conv(f32x4 (&acc)[H * W / 16], Frag<T> (&wa)[D], const T* const (&base)[6],
                                           const char* img, int PL, int HW, bool s2, const T* ra, const T* rb,
                                           int lane, const int (&py)[H * W / 16], const int (&px)[H * W / 16]) {
  using SS = ChainStream<C>;
  constexpr int FP = H * W / 16, ES = (int)sizeof(T), VE = 16 / ES;
  constexpr int Q0 = SS::S[SEG], NS3 = SS::N[SEG], NS = NS3 + (SEG == 4 ? SS::N[5] : 0), OFF = Q0 % D;
  const int g = lane >> 4, l16 = lane & 15;
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) acc[fp] = f32x4{0.f, 0.f, 0.f, 0.f};
  const T* cur = base[SEG];
  for (int j0 = 0; j0 < NS; j0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int s = j0 + d;
      if (s < NS) {
        Frag<T>& w = wa[(OFF + d) % D];
        Frag<T> bf[FP];
        if (s < NS3) {
          const int ck = s / 9, tap = s - 9 * ck, dy = tap / 3, dx = tap - 3 * dy;
          const char* pl = img + (ck * (32 / VE) + g * (ES / 2)) * PL;
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) {
            const int hy = s2 ? 2 * py[fp] + dy : py[fp] + dy, hx = s2 ? 2 * px[fp] + dx : px[fp] + dx;
            bf[fp] = load_planes<T>(pl + (hy * HW + hx) * 16, PL);
          }
        } else {                                         // res_conv chunk r of cat(ra, rb) at the pixel
          const int r = s - NS3, c0 = r * 32 + g * 8;
          const T* src = (c0 < C ? ra : rb) + (c0 < C ? c0 : c0 - C);
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) bf[fp] = load_frag<T>((const char*)(src + (fp * 16 + l16) * C));
        }
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) mfma_frag(acc[fp], w, bf[fp]);
        // refill with stream position Q0 + s + D: in this segment a plain offset, else the stream map
        w = s + D < NS3 ? load_frag<T>((const char*)(cur + (size_t)(s + D) * 512 + lane * 8))
                        : chain_frag<T, C>(base, Q0 + s + D, lane * 8);
      }
    }
  }
}

// epilogue: value = acc + add_b + add_t (+ identity residual `res`), stored as T to dst ([P][C]
// rows), channel statistics (mean, biased variance over the image) of the fp32 values into st
// (null: none), summed about the shift add_b + add_t
template <typename T, int C, int P>
__device__ __forceinline__ void chain_epilogue(const f32x4 (&acc)[P / 16], const float* add_b, const float* add_t,
                                               const T* res, T* dst, float* st, int co0, int lane) {
  constexpr int FP = P / 16;
  const int g = lane >> 4, l16 = lane & 15;
  float sh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int co = co0 + 4 * g + i;
    sh[i] = add_b[co] + (add_t ? add_t[co] : 0.f);
  }
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    const int p = fp * 16 + l16, co = co0 + 4 * g;
    float d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      d[i] = acc[fp][i] + (res ? to_f32<T>(res[p * C + co + i]) : 0.f);
      s1[i] += d[i];
      s2[i] += d[i] * d[i];
    }
    store4<T>(dst + p * C + co, d[0] + sh[0], d[1] + sh[1], d[2] + sh[2], d[3] + sh[3]);
  }
  if (st) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float t1 = row_sum16(s1[i]), t2 = row_sum16(s2[i]);
      if (l16 == 0) {
        const int co = co0 + 4 * g + i;
        const float m = t1 * (1.0f / P);
        st[co * 2] = sh[i] + m;
        st[co * 2 + 1] = fmaxf(t2 * (1.0f / P) - m * m, 0.f);
      }
    }
  }
}

// GroupNorm of the concat (stA | stB: per-channel mean, var over the image; Cin / groups channels
// per group) -> per-channel scale GS[c] / shift GS[2C + c]; fp32 combination of equal-count channel
// moments in a fixed order
template <int C, int NT>
__device__ __forceinline__ void chain_gn(int Cin, int groups, float eps, const float* stA, const float* stB,
                                         const float* gamma, const float* beta, float* GS) {
  const int cpg = Cin / groups;
  for (int c = threadIdx.x; c < Cin; c += NT) {
    const int c0 = c - c % cpg;
    float mg = 0.f;
    for (int k = 0; k < cpg; ++k) { const int cc = c0 + k; mg += (cc < C ? stA : stB)[(cc % C) * 2]; }
    mg *= 1.0f / cpg;
    float vg = 0.f;
    for (int k = 0; k < cpg; ++k) {
      const int cc = c0 + k;
      const float* e = (cc < C ? stA : stB) + (cc % C) * 2;
      const float dm = e[0] - mg;
      vg += e[1] + dm * dm;
    }
    vg *= 1.0f / cpg;
    const float rstd = 1.0f / sqrtf(vg + eps), sc = gamma[c] * rstd;
    GS[c] = sc;
    GS[2 * C + c] = beta[c] - mg * sc;
  }
}

// GroupNorm + SiLU of the raw concat (ra | rb) [P][C] into the interior of the zero-bordered
// plane-major image
template <typename T, int C, int H, int W, int NT, int PIMG>
__device__ __forceinline__ void chain_stage(int Cin, const T* ra, const T* rb, const float* GS, char* img) {
  constexpr int P = H * W, VE = 16 / (int)sizeof(T);
  const int nu = (Cin / VE) * P;
  for (int u = threadIdx.x; u < nu; u += NT) {
    const int q = u / P, p = u - q * P, c0 = q * VE;
    const T* src = (c0 < C ? ra : rb) + (p * C + (c0 < C ? c0 : c0 - C));   // (this form: clang 22 crashes on the pointer select)
    const f32x4 o = transform_lds<T>(*(const f32x4*)src, GS + c0, GS + 2 * C + c0);
    *(f32x4*)(img + q * PIMG + ((p / W + 1) * (W + 2) + (p % W + 1)) * 16) = o;
  }
}

template <typename T, int C, int H, int W>
__global__ __launch_bounds__(4 * C, 1) void conv_chain_kernel(ChainArgs a) {
  using G = ChainGeo<T, C, H, W>;
  constexpr int P = G::P, FP = G::FP, NT = G::NT, VE = G::VE, ES = G::ES;
  constexpr int D = SDDM_CHAIN_RING;                     // weight-fragment ring depth (K steps in flight)
  static_assert(P % 16 == 0 && C % 32 == 0 && G::LDS <= kLdsBytes && NT == 4 * C, "chain geometry");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* IN = smem;                                       // downs.10 halo, then IMG (alias)
  char* IMG = smem;
  T* RD = (T*)(smem + G::OFF_RD);                        // downs.10 output (raw, [P][C])
  T* RH = (T*)(smem + G::OFF_RH);                        // mid.0.block1 / ups.0.block1 output
  T* RM = (T*)(smem + G::OFF_RM);                        // mid.0.block2 output
  float* ST = (float*)(smem + G::OFF_ST);                // statistics: 0 D10, 1 H1, 2 M, 3 H2
  float* GS = (float*)(smem + G::OFF_GS);                // scale [2C], shift [2C]
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, l16 = lane & 15;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int co0 = wv * 16;                               // this wave's output channels
  const int t_step = a.t_dev ? *a.t_dev : 0;
  const int trow = a.temb_per_b ? b : t_step;
  const float* temb0 = a.temb[0] ? a.temb[0] + (size_t)trow * a.temb_ld : nullptr;
  const float* temb1 = a.temb[1] ? a.temb[1] + (size_t)trow * a.temb_ld : nullptr;

  // ---- downs.10 input halo: rows -1 .. 2H-1, cols -1 .. 2W-1 of the level's input ----
  {
    constexpr int NU = (C / VE) * G::HI * G::WI, UPT = (NU + NT - 1) / NT;
    const char* src = (const char*)a.x + (size_t)b * (2 * H) * (2 * W) * C * ES;
    f32x4 v[UPT];
#pragma unroll
    for (int k = 0; k < UPT; ++k) {                      // every load before the first store
      const int u = min(tid + k * NT, NU - 1), q = u / (G::HI * G::WI), hp = u - q * (G::HI * G::WI);
      const int iy = hp / G::WI - 1, ix = hp % G::WI - 1;
      const bool ok = iy >= 0 && ix >= 0;
      v[k] = *(const f32x4*)(src + (ok ? ((iy * (2 * W) + ix) * C + q * VE) * ES : 0));
      if (!ok) v[k] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int u = tid + k * NT;
      if (u < NU) {
        const int q = u / (G::HI * G::WI), hp = u - q * (G::HI * G::WI);
        *(f32x4*)(IN + q * G::PIN + hp * 16) = v[k];
      }
    }
  }
  __syncthreads();

  int py[FP], px[FP];                                    // pixel of each of this lane's fragments
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) { const int p = fp * 16 + l16; py[fp] = p / W; px[fp] = p % W; }
  f32x4 acc[FP];
  // the wave's weight stream: segment k's first fragment of output-channel block wv, lane piece
  using SS = ChainStream<C>;
  const T* base[6];
#pragma unroll
  for (int k = 0; k < 6; ++k)
    base[k] = (const T*)(k < 5 ? a.wgt[k] : a.res_wgt) + ((size_t)wv * SS::N[k]) * 512;
  Frag<T> wa[D];
#pragma unroll
  for (int d = 0; d < D; ++d) wa[d] = chain_frag<T, C>(base, d, lane * 8);
  // 1. downs.10: stride-2 conv of the raw input (no GroupNorm)
  chain_conv<T, C, H, W, D, 0>(acc, wa, base, IN, G::PIN, G::WI, true, nullptr, nullptr, lane, py, px);
  chain_epilogue<T, C, P>(acc, a.bias[0], nullptr, nullptr, RD, ST + 0 * 2 * C, co0, lane);
  __syncthreads();                                       // IN dead, RD / its statistics visible
  for (int u = tid; u < G::IMG_BYTES / 16; u += NT) *(f32x4*)(IMG + u * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
  chain_gn<C, NT>(C, a.groups, a.eps, ST + 0 * 2 * C, nullptr, a.gamma[0], a.beta[0], GS);
  __syncthreads();
  // 2. mid.0.block1: GN+SiLU(D10) -> conv + bias + noise embedding
  chain_stage<T, C, H, W, NT, G::PIMG>(C, RD, nullptr, GS, IMG);
  __syncthreads();
  chain_conv<T, C, H, W, D, 1>(acc, wa, base, IMG, G::PIMG, G::WP, false, nullptr, nullptr, lane, py, px);
  chain_epilogue<T, C, P>(acc, a.bias[1], temb0, nullptr, RH, ST + 1 * 2 * C, co0, lane);
  __syncthreads();
  chain_gn<C, NT>(C, a.groups, a.eps, ST + 1 * 2 * C, nullptr, a.gamma[1], a.beta[1], GS);
  __syncthreads();
  // 3. mid.0.block2: GN+SiLU(H1) -> conv + bias + identity residual (D10)
  chain_stage<T, C, H, W, NT, G::PIMG>(C, RH, nullptr, GS, IMG);
  __syncthreads();
  chain_conv<T, C, H, W, D, 2>(acc, wa, base, IMG, G::PIMG, G::WP, false, nullptr, nullptr, lane, py, px);
  chain_epilogue<T, C, P>(acc, a.bias[2], nullptr, RD, RM, ST + 2 * 2 * C, co0, lane);
  __syncthreads();
  chain_gn<C, NT>(2 * C, a.groups, a.eps, ST + 2 * 2 * C, ST + 0 * 2 * C, a.gamma[2], a.beta[2], GS);
  __syncthreads();
  // 4. ups.0.block1: GN+SiLU(cat(M, D10)) -> conv + bias + noise embedding
  chain_stage<T, C, H, W, NT, G::PIMG>(2 * C, RM, RD, GS, IMG);
  __syncthreads();
  chain_conv<T, C, H, W, D, 3>(acc, wa, base, IMG, G::PIMG, G::WP, false, nullptr, nullptr, lane, py, px);
  chain_epilogue<T, C, P>(acc, a.bias[3], temb1, nullptr, RH, ST + 3 * 2 * C, co0, lane);
  __syncthreads();
  chain_gn<C, NT>(C, a.groups, a.eps, ST + 3 * 2 * C, nullptr, a.gamma[3], a.beta[3], GS);
  __syncthreads();
  // 5. ups.0.block2: GN+SiLU(H2) -> conv + bias (with the res_conv bias) + res_conv(cat(M, D10))
  chain_stage<T, C, H, W, NT, G::PIMG>(C, RH, nullptr, GS, IMG);
  __syncthreads();
  chain_conv<T, C, H, W, D, 4>(acc, wa, base, IMG, G::PIMG, G::WP, false, RM, RD, lane, py, px);
  chain_epilogue<T, C, P>(acc, a.bias[4], nullptr, nullptr, (T*)a.out + (size_t)b * P * C, nullptr, co0, lane);
}

hipError_t launch_conv_chain(int dtype, const ChainArgs& a, int B, hipStream_t s) {
  if (a.C != 160 || a.H != 8 || a.W != 4 || a.groups <= 0 || (2 * a.C) % a.groups || a.C % a.groups) return hipErrorInvalidValue;
  if (dtype == DT_BF16) {
    using G = ChainGeo<bf16_t, 160, 8, 4>;
    hipLaunchKernelGGL((conv_chain_kernel<bf16_t, 160, 8, 4>), dim3(B), dim3(G::NT), G::LDS, s, a);
  } else if (dtype == DT_F16) {
    using G = ChainGeo<f16_t, 160, 8, 4>;
    hipLaunchKernelGGL((conv_chain_kernel<f16_t, 160, 8, 4>), dim3(B), dim3(G::NT), G::LDS, s, a);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace sddm
