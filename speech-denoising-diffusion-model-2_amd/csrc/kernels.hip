// Device kernels of the MI355X-native SDDM sampler (gfx950 / CDNA4, wave64).
//
// One reverse-diffusion step of SDDM.infer (model/model.py:106-122) with UNetModified2 is
//   conv_in (framing + Conv2d 2->32, stats)                    UNetModified2.py:244-247,177
//   for every GroupNorm: gn_finalize (per-tile stats -> scale/shift)
//   conv3x3 (MFMA implicit GEMM, prologue GN+SiLU / upsample / virtual concat,
//            epilogue bias + noise embedding + residual (identity or fused 1x1) + tile stats)
//   final (GN+SiLU -> Conv 32->1 -> overlapAdd -> p_transition with Philox noise)
// Activations are NHWC ([B][frames][segment][C]) so a pixel's channels are contiguous and
// the MFMA K dimension (tap, channel) reads 16-byte vectors straight from LDS.
#include "sddm_common.h"
#include "kernels.h"
#include "conv_common.h"
#include <algorithm>
#include <type_traits>

namespace sddm {


// =============================================================================================
// Noise-level embedding: PositionalEncoding -> Linear -> Swish -> Linear -> Swish
// (UNetModified2.py:49-68,168-174) and every ResnetBlock's FeatureWiseAffine Linear
// (UNetModified2.py:72-89) with the following conv's bias folded in.  One block per row.
// =============================================================================================
__global__ __launch_bounds__(256) void embed_kernel(EmbedArgs a) {
  __shared__ float enc[128];
  __shared__ float h1[512];
  __shared__ float h2[128];
  const int r = blockIdx.x, tid = threadIdx.x, D = a.dim, H = a.dim / 2, D4 = 4 * a.dim;
  float nl;
  if (a.noise_levels) nl = a.noise_levels[r];
  else if (a.time_step_mode) nl = (float)r;
  else nl = a.table[r];
  if (tid < D) {
    // encoding = diffusion_step * embedding_vector (fp32 product), then accurate sin / cos
    const float arg = __fmul_rn(nl, a.emb_vec[tid % H]);
    enc[tid] = tid < H ? sinf(arg) : cosf(arg);
  }
  __syncthreads();
  for (int j = tid; j < D4; j += blockDim.x) {
    float s = a.b1[j];
    for (int k = 0; k < D; ++k) s += a.w1[j * D + k] * enc[k];
    h1[j] = s / (1.0f + expf(-s));
  }
  __syncthreads();
  for (int i = tid; i < D; i += blockDim.x) {
    float s = a.b2[i];
    for (int j = 0; j < D4; ++j) s += a.w2[i * D4 + j] * h1[j];
    h2[i] = s / (1.0f + expf(-s));
  }
  __syncthreads();
  for (int c = tid; c < a.SC; c += blockDim.x) {
    float s = a.pb[c];
    for (int i = 0; i < D; ++i) s += a.pw[c * D + i] * h2[i];
    a.out[(size_t)r * a.SC + c] = s;
  }
}

hipError_t launch_embed(const EmbedArgs& a, hipStream_t s) {
  if (a.dim > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(embed_kernel, dim3(a.R), dim3(256), 0, s, a);
  return hipGetLastError();
}

// =============================================================================================
// GroupNorm finalize: per-tile (sum, M2) of each channel -> per-(b, channel) scale and shift.
// Chan's parallel combination in fp64, two deterministic passes (no atomics).
// =============================================================================================
__device__ __forceinline__ double block_sum_d(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

__global__ __launch_bounds__(256) void gn_finalize_kernel(GNArgs a) {
  __shared__ double red[8];
  const int g = blockIdx.x, b = blockIdx.y;
  const int C = a.a.C + a.b.C, cpg = C / a.G;
  const int c_begin = g * cpg;
  double s = 0.0;
  for (int cc = 0; cc < cpg; ++cc) {
    const int c = c_begin + cc;
    const GNSrc& src = c < a.a.C ? a.a : a.b;
    const int ci = c < a.a.C ? c : c - a.a.C;
    const float* st = src.stats + ((size_t)b * src.tiles * src.C + ci) * 2;
    for (int t = threadIdx.x; t < src.tiles; t += blockDim.x) s += (double)st[(size_t)t * src.C * 2];
  }
  const double S = block_sum_d(s, red);
  double ntot = 0.0;
  for (int cc = 0; cc < cpg; ++cc) {
    const int c = c_begin + cc;
    const GNSrc& src = c < a.a.C ? a.a : a.b;
    ntot += (double)src.tiles * src.n_tile;
  }
  const double mean = S / ntot;
  double m2 = 0.0;
  for (int cc = 0; cc < cpg; ++cc) {
    const int c = c_begin + cc;
    const GNSrc& src = c < a.a.C ? a.a : a.b;
    const int ci = c < a.a.C ? c : c - a.a.C;
    const float* st = src.stats + ((size_t)b * src.tiles * src.C + ci) * 2;
    const double nt = (double)src.n_tile;
    for (int t = threadIdx.x; t < src.tiles; t += blockDim.x) {
      const double ts = st[(size_t)t * src.C * 2], tm2 = st[(size_t)t * src.C * 2 + 1];
      const double d = ts / nt - mean;
      m2 += tm2 + nt * d * d;
    }
  }
  const double M2 = block_sum_d(m2, red);
  const double rstd = 1.0 / sqrt(M2 / ntot + (double)a.eps);
  for (int cc = threadIdx.x; cc < cpg; cc += blockDim.x) {
    const int c = c_begin + cc;
    const double sc = (double)a.gamma[c] * rstd;
    a.scale[(size_t)b * C + c] = (float)sc;
    a.shift[(size_t)b * C + c] = (float)((double)a.beta[c] - mean * sc);
  }
}

hipError_t launch_gn_finalize(const GNArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(gn_finalize_kernel, dim3(a.G, a.B), dim3(256), 0, s, a);
  return hipGetLastError();
}

// =============================================================================================
// conv_in: SignalToFrames on cond and x_t (idx[f,w] = S*f + w), channel concat, Conv2d(2, 32, 3,
// pad 1) + bias, as an MFMA over K = 18 taps (2 signals x 3x3, zero-padded to the MFMA depth).
// The block's sample window of both signals is staged in LDS once (two coalesced loads per
// thread); the framing gathers then read LDS.  T = float: exact f32 MFMA (16x16x4, K = 20);
// bf16 / f16 storage: fp16 hi/lo split of both operands (x*w = xh*wh + xh*wl + xl*wh, error
// ~2^-22 relative) so the fp32 signal keeps fp32 accuracy.  A block = TR frame rows x W = 512
// pixels, a wave = 8 fragments of 16 pixels.  Tile statistics are reduced from registers.
// =============================================================================================
template <typename T>
__global__ __launch_bounds__(256) void conv_in_kernel(ConvInArgs a) {
  constexpr int CO = 32;                    // inner_channel (checked by the launcher)
  constexpr int IMAX = 6 * 130;             // (TR + 2) x (W + 2) frame image per signal (checked by the launcher)
  constexpr int NFR = 8;                    // pixel fragments per wave (512 pixels per block)
  __shared__ float img[2][IMAX];            // zero-bordered frames f0-1 .. f0+TR of cond and x_t
  __shared__ float xs_red[4][CO][2];        // per-wave channel sums for the tile statistics
  const int b = blockIdx.y, f0 = blockIdx.x * a.TR, tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  if (a.t_dev && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) *a.t_dev -= 1;
  SDDM_STAMP_AT(a, 0, blockIdx.x + blockIdx.y * (a.F / a.TR));
  const int S = a.S, F = a.F, W = a.W, IW = W + 2, IH = a.TR + 2;
  // bias and weights first: issued before the frame image loads, so their round trip overlaps
  // the image's instead of following it (stamps: the staging phase was two round trips, 4.5 us)
  constexpr int KPL = sizeof(T) == 4 ? 5 : 8;   // K values per lane per pixel fragment
  float bias[2][4];
#pragma unroll
  for (int fc = 0; fc < 2; ++fc)
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[fc][i] = a.bias[fc * 16 + 4 * g + i];
  float wf[2][KPL];                             // weights as MFMA A operands (rows = output channels)
#pragma unroll
  for (int j = 0; j < KPL; ++j) {
    const int k = sizeof(T) == 4 ? 4 * j + g : 8 * g + j;
    const int kk = k < 18 ? k : 0;              // (clamped: unconditional loads, masked below)
#pragma unroll
    for (int fc = 0; fc < 2; ++fc) wf[fc][j] = a.w[(fc * 16 + (lane & 15)) * 18 + kk];
  }
  {  // every load of the frame image issued before the first is stored (clamped addresses:
     // a load under a condition is waited for at the branch join)
    const float* c0 = a.cond + (size_t)b * a.N;
    const float* x0 = a.x + (size_t)b * a.N;
    constexpr int IPT = (IMAX + 255) / 256;
    float cv[IPT], xv[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = min(tid + 256 * k, IH * IW - 1);
      const int r = i / IW, c = i - r * IW, f = f0 - 1 + r, w = c - 1;
      const bool ok = f >= 0 && f < F && w >= 0 && w < W;
      const int n = ok ? f * S + w : 0;
      cv[k] = c0[n];
      xv[k] = x0[n];
      cv[k] = ok ? cv[k] : 0.f;
      xv[k] = ok ? xv[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const int i = tid + 256 * k;
      if (i < IH * IW) { img[0][i] = cv[k]; img[1][i] = xv[k]; }
    }
  }
  // this lane's K entries k -> (signal, dy, dx) as offsets into the frame image (k >= 18: zero)
  int koff[KPL];
  bool kok[KPL];
#pragma unroll
  for (int j = 0; j < KPL; ++j) {
    const int k = sizeof(T) == 4 ? 4 * j + g : 8 * g + j;
    kok[j] = k < 18;
    const int kk = kok[j] ? k : 0, ch = kk >= 9 ? 1 : 0, tap = kk - 9 * ch;
    koff[j] = ch * IMAX + (tap / 3) * IW + (tap % 3);
#pragma unroll
    for (int fc = 0; fc < 2; ++fc) wf[fc][j] = kok[j] ? wf[fc][j] : 0.f;
  }
  f16x8 wh[2], wl[2];
#pragma unroll
  for (int fc = 0; fc < 2; ++fc)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = j < KPL ? wf[fc][j] : 0.f;
      wh[fc][j] = (f16_t)v;
      wl[fc][j] = (f16_t)(v - (float)wh[fc][j]);
    }
  f32x2 st1[2][2], st2[2][2], bp[2][2];                  // packed pairs (accumulator register pairs)
#pragma unroll
  for (int fc = 0; fc < 2; ++fc)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      st1[fc][h] = f32x2{0.f, 0.f};
      st2[fc][h] = f32x2{0.f, 0.f};
      bp[fc][h] = f32x2{bias[fc][2 * h], bias[fc][2 * h + 1]};
    }
  const float rW = 1.0f / (float)W;
  __syncthreads();                                        // frame image staged
  SDDM_STAMP_AT(a, 1, blockIdx.x + blockIdx.y * (a.F / a.TR));
  const float* imgf = &img[0][0];
#pragma unroll 2
  for (int fr = 0; fr < NFR; ++fr) {
    const int p = wave * (NFR * 16) + fr * 16 + (lane & 15);
    const int r = fdivi(p, rW), w = p - r * W;
    const int pb = r * IW + w;                              // image index of tap (0, 0)
    float xv[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) xv[j] = kok[j] ? imgf[pb + koff[j]] : 0.f;
    f32x4 acc[2];
    if constexpr (sizeof(T) == 4) {                          // exact fp32 MFMA
#pragma unroll
      for (int fc = 0; fc < 2; ++fc) {
        acc[fc] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < KPL; ++j) acc[fc] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[fc][j], xv[j], acc[fc], 0, 0, 0);
      }
    } else if constexpr (std::is_same<T, bf16_t>::value) {  // bf16 storage: fp16 operands (2^-11 << 2^-8)
      f16x8 xh;
#pragma unroll
      for (int j = 0; j < 8; ++j) xh[j] = (f16_t)(j < KPL ? xv[j] : 0.f);
#pragma unroll
      for (int fc = 0; fc < 2; ++fc)
        acc[fc] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[fc], xh, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    } else {                                                  // f16 storage: hi/lo split (fp32-accurate)
      f16x8 xh, xl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = j < KPL ? xv[j] : 0.f;
        xh[j] = (f16_t)v;
        xl[j] = (f16_t)(v - (float)xh[j]);
      }
#pragma unroll
      for (int fc = 0; fc < 2; ++fc) {
        acc[fc] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[fc], xh, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        acc[fc] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[fc], xl, acc[fc], 0, 0, 0);
        acc[fc] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[fc], xh, acc[fc], 0, 0, 0);
      }
    }
    T* op = (T*)a.out + (((size_t)b * F + f0 + r) * W + w) * CO;
#pragma unroll
    for (int fc = 0; fc < 2; ++fc) {
      // statistics of the fp32 values about the shift = bias (common to the whole tile)
      const f32x2 d0 = f32x2{acc[fc][0], acc[fc][1]}, d1 = f32x2{acc[fc][2], acc[fc][3]};
      st1[fc][0] += d0;
      st1[fc][1] += d1;
      st2[fc][0] = __builtin_elementwise_fma(d0, d0, st2[fc][0]);
      st2[fc][1] = __builtin_elementwise_fma(d1, d1, st2[fc][1]);
      store4p<T>(op + fc * 16 + 4 * g, d0 + bp[fc][0], d1 + bp[fc][1]);
    }
  }
  SDDM_STAMP_AT(a, 2, blockIdx.x + blockIdx.y * (a.F / a.TR));
  // tile statistics: lanes of one channel group (xor 1..8) -> 4 waves (LDS), plain sums about the bias
#pragma unroll
  for (int fc = 0; fc < 2; ++fc)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float t1 = row_sum16(st1[fc][i >> 1][i & 1]);    // DPP row adds (VALU)
      const float t2 = row_sum16(st2[fc][i >> 1][i & 1]);
      if ((lane & 15) == 0) {
        xs_red[wave][fc * 16 + 4 * g + i][0] = t1;
        xs_red[wave][fc * 16 + 4 * g + i][1] = t2;
      }
    }
  lds_sync();                                              // (the output stores stay in flight)
  SDDM_STAMP_AT(a, 3, blockIdx.x + blockIdx.y * (a.F / a.TR));
  if (tid < CO) {
    const float n = (float)(a.TR * W);
    float S1 = 0.f, S2 = 0.f;
#pragma unroll
    for (int w4 = 0; w4 < 4; ++w4) { S1 += xs_red[w4][tid][0]; S2 += xs_red[w4][tid][1]; }
    float* dst = a.stats + (((size_t)b * (a.F / a.TR) + blockIdx.x) * CO + tid) * 2;
    dst[0] = a.bias[tid] * n + S1;                 // sum
    dst[1] = fmaxf(S2 - S1 * S1 / n, 0.f);        // M2 about the tile mean
  }
  SDDM_STAMP_AT(a, 6, blockIdx.x + blockIdx.y * (a.F / a.TR));
  SDDM_STAMP_AT(a, 7, blockIdx.x + blockIdx.y * (a.F / a.TR));
}

hipError_t launch_conv_in(int dtype, const ConvInArgs& a, int B, hipStream_t s) {
  if (a.Cout != 32 || a.TR * a.W != 512 || a.F % a.TR || (a.TR + 2) * (a.W + 2) > 6 * 130) return hipErrorInvalidValue;
  dim3 grid(a.F / a.TR, B);
  if (dtype == DT_F32) hipLaunchKernelGGL(conv_in_kernel<float>, grid, dim3(256), 0, s, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(conv_in_kernel<bf16_t>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(conv_in_kernel<f16_t>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// =============================================================================================
// Transitions (diffusion.py:164-223).  Operation order and rounding follow the reference:
// no FMA contraction in this region.
// =============================================================================================
#pragma clang fp contract(off)
__device__ __forceinline__ float transition_one(int mode, const TransCoef& c, int t, float xt, float e,
                                                float cond, float z) {
  float x;
  if (mode == 4) mode = 0;                                       // condition_in uses p_transition
  if (mode == 0 || mode == 1) {                                  // original / condition_in / sr3
    x = (xt - c.pnc[t] * e) / sqrtf(c.alphas[t]);
    if (t > 1) x = x + (mode == 0 ? c.sigma[t] : sqrtf(c.betas[t])) * z;
  } else if (mode == 2) {                                        // supportive (diffusion.py:203-208)
    const float g = c.sgamma[t];
    const float mu = xt - c.pnc[t] * e;
    x = ((1.0f - g) * mu + g * cond) / sqrtf(c.alphas[t]);
    if (t > 1) x = x + fmaxf(0.0f, c.ssh[t]) * z;
  } else {                                                       // conditional (diffusion.py:216-221)
    x = c.c_xt[t] * xt + c.c_yt[t] * cond - c.c_epst[t] * e;
    if (t > 1) x = x + c.sde[t] * z;
  }
  return clamp_pm1(x);
}

__global__ __launch_bounds__(256) void transition_kernel(TransArgs a) {
  const int t = a.t_dev ? *a.t_dev : a.t;
  const bool needs_cond = a.mode >= 2;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.total; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = (uint64_t)(a.row_offset * a.N + i);
    const float z = t > 1 ? (a.noise ? a.noise[(int64_t)t * a.noise_ld + i] : philox_normal1(a.seed, (uint32_t)t, e)) : 0.f;
    a.out[i] = transition_one(a.mode, a.co, t, a.x_t[i], a.eps[i], needs_cond ? a.cond[i] : 0.f, z);
  }
}

__global__ __launch_bounds__(256) void init_state_kernel(InitArgs a) {
  const int T = a.T;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.total; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t e = (uint64_t)(a.row_offset * (int64_t)a.N + i);
    float v;
    if (a.mode == 2) {
      v = a.cond[i];                                              // supportive: x_T = condition
    } else {
      const float z = a.noise ? a.noise[i] : philox_normal1(a.seed, 0u, e);
      if (a.mode == 4) {                                          // condition_in: get_x_T
        const float s = a.co.sqrt_alpha_bar[T];
        v = s * a.cond[i] + sqrtf(1.0f - s * s) * z;
      } else if (a.mode == 3) {                                   // conditional: get_x_T_conditional
        v = a.co.sqrt_alpha_bar[T] * a.cond[i] + a.co.sqrt_delta[T] * z;
      } else {
        v = z;                                                    // original / sr3: randn_like
      }
    }
    a.out[i] = v;
  }
}

#pragma clang fp contract(fast)

// =============================================================================================
// Final Block (GN+SiLU -> Conv 3x3 C->1) + overlapAdd + transition, fused.  A block owns frames
// [f0, f0+FT) and the samples [S*f0, S*(f0+FT)) (the last block also the tail up to N).
//  phase 1: every input pixel of rows [f0-back-1, f0+FT] -> its 9 per-tap partial dot products
//           P[tap] = sum_c w[c][tap] * silu(gn(x[c])) (each pixel transformed once), in LDS;
//  phase 2: y[f][w] = bias + sum_taps P[tap][f+dy-1][w+dx-1] for frames [f0-back, f0+FT);
//  phase 3: overlapAdd in ascending frame order (UNetModified2.py:37-39) and p_transition, four
//           consecutive samples per thread (one Philox counter group).
// =============================================================================================
// compile-time geometry of the final block (FinalShape: frames per block, segment, hop, frames,
// samples, channels) and transition mode (kFinalModeArg: from FinalArgs) for the headline
// workload; other lengths run the generic instantiation (SH = 0)
struct FinalShape { int FT, W, S, F, N, C, GT, GNT, G; };   // GroupNorm source tiles, pixels per tile, groups
static constexpr FinalShape kFinalShapes[] = {
    {1, 1, 1, 1, 1, 1, 1, 1, 1},                   // generic (fields unused)
    {8, 128, 64, 256, 16448, 32, 16, 2048, 32},    // UNetModified2 config_unet.json, 16448 samples
};
static constexpr int kNFinalShapes = (int)(sizeof(kFinalShapes) / sizeof(kFinalShapes[0]));
constexpr int kFinalModeArg = -99;

template <typename T, int NT, int SH, int MODE>
__global__ __launch_bounds__(NT) void final_kernel(FinalArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NWV = NT / 64;                // waves per block
  constexpr FinalShape FS = kFinalShapes[SH];
  constexpr bool CS = SH > 0;
  const int FT = CS ? FS.FT : a.FT, Ns = CS ? FS.N : a.N;
  const int mode = MODE != kFinalModeArg ? MODE : a.mode;
  const int C = CS ? FS.C : a.C, W = CS ? FS.W : a.W, S = CS ? FS.S : a.S, F = CS ? FS.F : a.F;
  // frame tile and image: a 1-D grid is dealt to the XCDs in the order of xcd_block (the frame
  // tiles of an image on one XCD, so the halo frames a tile shares with its neighbours come from
  // that XCD's L2); a 2-D grid is (tile, image)
  int ftile, b;
  if (gridDim.y == 1) {
    int zz;
    xcd_block<true>(F / FT, 1, ftile, b, zz);
  } else {
    ftile = blockIdx.x; b = blockIdx.y;
  }
  const int f0 = ftile * FT, tid = threadIdx.x;
  const int back = W / S - 1;                 // extra frames before f0 needed by the OLA
  const int YR = FT + back;                   // y rows: frames [f0-back, f0+FT)
  const int PR = YR + 2, PC = W + 2;          // partial-product rows / cols (zero halo cols)
  float* P = (float*)smem;                    // [9][PR][PC]
  float* y = P + 9 * PR * PC;                 // [YR][W]
  float* gs = y + YR * W;                     // [2][C]
  SDDM_STAMP_AT(a, 0, ftile + b * (F / FT));
  // every independent load first: the transition's x_t / condition (one 4-sample vector per
  // thread: the block's samples fit one pass, checked by the launcher), the GroupNorm statistics
  // and the first pass of activation fragments; then one wait
  const int n_begin = f0 * S;
  const int n_end = (f0 + FT >= F) ? Ns : (f0 + FT) * S;
  float* xrow = a.x + (size_t)b * Ns;
  const float* crow = a.cond ? a.cond + (size_t)b * Ns : xrow;
  const int n4 = n_begin + 4 * tid;
  const int n4c = n4 < n_end ? n4 : n_begin;
  const f32x4 xin = *(const f32x4*)(xrow + n4c);
  const f32x4 cin = *(const f32x4*)(crow + n4c);
  const GNFuse gf{a.gst, CS ? FS.GT : a.gtiles, CS ? FS.GNT : a.gntile, nullptr, 0, 0, a.gamma, a.beta, CS ? FS.G : a.groups, a.eps};
  GNLoad gl;
  gl.issue(gf, b, C, 0, true, a.gamma);
  // phase 1 as an MFMA: P[tap][pos] = sum_c w[c][tap] * silu(gn(x[c][pos])) with A = the 9 taps
  // (rows, padded to 16) x 32 channels and B = 32 channels x 16 positions.  bf16 / f16: fp16
  // hi/lo split of both operands (fp32-accurate products); float: exact f32 MFMA.
  const int lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const T* src = (const T*)a.src + (size_t)b * F * W * C;
  const int tapr = lane & 15;
  const int npos = PR * PC, nfr = (npos + 15) / 16;
  // every fragment of this wave is loaded before the first is used (one memory latency, not one
  // per fragment): FRW fragments per pass
  constexpr int FRW = 12;                            // fragments per wave and pass
  constexpr int NV = (int)sizeof(T) * 8 / 16;        // 16-byte vectors per 8 channels
  typedef T vec8 __attribute__((ext_vector_type(8)));
  f32x4 xr[FRW][NV];
  unsigned inmask = 0;                               // bit q: fragment q's position is inside the image
  const float rPC = 1.0f / (float)PC;                // positions < 2^21: fdivi is exact
  auto load_pass = [&](int fr0) {
    inmask = 0;
#pragma unroll
    for (int q = 0; q < FRW; ++q) {
      const int pp = (fr0 + NWV * q) * 16 + (lane & 15);
      const int r = fdivi(pp, rPC), col = pp - r * PC;
      const int f = f0 - back - 1 + r, w = col - 1;
      const bool in = pp < npos && f >= 0 && f < F && w >= 0 && w < W;
      inmask |= in ? 1u << q : 0u;
      const int off = in ? (f * W + w) * C + 8 * g : 8 * g;   // < 2^31 elements per image
#pragma unroll
      for (int h = 0; h < NV; ++h) xr[q][h] = *(const f32x4*)((const char*)(src + off) + 16 * h);
    }
  };
  load_pass(wave);
  // the conv weights of this lane's 8 channels, before the GroupNorm wait (one round trip, not two)
  float wraw[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) wraw[j] = a.w[(8 * g + j) * 9 + (tapr < 9 ? tapr : 0)];
  gl.finish(gf, b, C, 0, gs, gs + C);
  lds_sync();                                        // scale / shift visible (loads stay in flight)
  SDDM_STAMP_AT(a, 1, ftile + b * (F / FT));
  // SiLU through exp2 with the constants folded: t = -(x sc + sh) log2(e) = x sc' + sh', and
  // silu = -ln2 * t / (1 + 2^t); the -ln2 goes into the fp32 weights (one multiply per lane)
  constexpr float kL2E = 1.4426950408889634f, kLN2 = 0.6931471805599453f;
  float wv[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = 8 * g + j;
    wv[j] = tapr < 9 ? wraw[j] * -kLN2 : 0.f;
    sc[j] = gs[c] * -kL2E;
    sh[j] = gs[C + c] * -kL2E;
  }
  for (int fr0 = wave; fr0 < nfr; fr0 += NWV * FRW) {
  if (fr0 != wave) load_pass(fr0);                   // inputs larger than one pass
#pragma unroll
  for (int q = 0; q < FRW; ++q) {
    const int fr = fr0 + NWV * q;
    const int pp = fr * 16 + (lane & 15);
    const int r = fdivi(pp, rPC), col = pp - r * PC;
    const bool in = (inmask >> q) & 1u;               // zero padding: the position's column of the
    const vec8 x = __builtin_bit_cast(vec8, xr[q]);   // product is masked, not its 8 inputs
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const f32x2 t = __builtin_elementwise_fma(f32x2{to_f32<T>(x[j]), to_f32<T>(x[j + 1])}, f32x2{sc[j], sc[j + 1]},
                                                f32x2{sh[j], sh[j + 1]});
      const f32x2 d = f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + f32x2{1.f, 1.f};
      const f32x2 o = t * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
      v[j] = o.x;
      v[j + 1] = o.y;
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if constexpr (sizeof(T) == 4) {
      const Frag<float> A{f32x4{wv[0], wv[1], wv[2], wv[3]}, f32x4{wv[4], wv[5], wv[6], wv[7]}};
      const Frag<float> Bf{f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}};
      mfma_frag(acc, A, Bf);
    } else {
      f16x8 wh, wl, xh, xl;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        wh[j] = (f16_t)wv[j]; wl[j] = (f16_t)(wv[j] - (float)wh[j]);
        xh[j] = (f16_t)v[j];  xl[j] = (f16_t)(v[j] - (float)xh[j]);
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xh, acc, 0, 0, 0);
      if constexpr (!std::is_same<T, bf16_t>::value) {   // bf16 storage: the fp16 products suffice
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, xh, acc, 0, 0, 0);
      }
    }
    // a lane's MFMA output column is its own position (lane & 15), all taps of it: padding
    // positions store 0 (outside the image), positions past the halo store nothing
    if (fr < nfr && pp < npos)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (4 * g + i < 9) P[((4 * g + i) * PR + r) * PC + col] = in ? acc[i] : 0.f;
  }
  }
  lds_sync();
  SDDM_STAMP_AT(a, 2, ftile + b * (F / FT));
  for (int p = tid; p < YR * W; p += NT) {
    const int r = p / W, w = p - r * W;        // y row r <-> P rows r .. r+2, cols w .. w+2
    float s = 0.f;
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) s += P[((dy * 3 + dx) * PR + r + dy) * PC + w + dx];
    y[p] = s + a.bias;
  }
  lds_sync();
  SDDM_STAMP_AT(a, 3, ftile + b * (F / FT));
  const int t = a.t_dev ? *a.t_dev : 0;
  const uint64_t seed = a.sp ? a.sp->seed : a.seed;
  const int64_t row_offset = a.sp ? a.sp->row_offset : a.row_offset;
  const int64_t ebase = (row_offset + b) * (int64_t)Ns;
  if (n4 < n_end) {
    const uint64_t e0 = (uint64_t)(ebase + n4);
    f32x4 z = {0.f, 0.f, 0.f, 0.f};
    const bool aligned = (e0 & 3) == 0;
    if (mode >= 0 && t > 1 && a.noise) z = *(const f32x4*)(a.noise + (int64_t)t * a.noise_ld + (int64_t)b * Ns + n4);
    else if (mode >= 0 && t > 1 && aligned) z = philox_normal4(seed, (uint32_t)t, e0 >> 2);
    f32x4 e4 = {0.f, 0.f, 0.f, 0.f};
    if ((S & 3) == 0 && (W & 3) == 0) {
      // overlapAdd of 4 consecutive samples: with S and W multiples of 4 they are covered by the
      // same frames [flo, fhi], so the frame range is computed once (float-reciprocal division,
      // n4 < 2^21) and each frame contributes one 16-byte LDS read; ascending frame order as
      // UNetModified2.py:37-39
      const float rS = 1.0f / (float)S;
      const int fhi = min(F - 1, fdivi(n4, rS));
      const int flo = n4 - W + 1 <= 0 ? 0 : fdivi(n4 - W + S, rS);
      for (int f = flo; f <= fhi; ++f) e4 += *(const f32x4*)(y + (f - (f0 - back)) * W + (n4 - f * S));
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n4 + j;
        int flo = (n - W + S) / S;
        if (n - W + 1 <= 0) flo = 0;
        const int fhi = min(F - 1, n / S);
        float e = 0.f;
        for (int f = flo; f <= fhi; ++f) e += y[(f - (f0 - back)) * W + (n - f * S)];
        e4[j] = e;
      }
    }
    if (mode < 0) {
      if (n4 + 3 < n_end) *(f32x4*)(a.eps_out + (size_t)b * Ns + n4) = e4;
      else
        for (int j = 0; j < 4 && n4 + j < n_end; ++j) a.eps_out[(size_t)b * Ns + n4 + j] = e4[j];
    } else {
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float zz = (t > 1) ? ((aligned || a.noise) ? z[j] : philox_normal1(seed, (uint32_t)t, e0 + j)) : 0.f;
        o[j] = transition_one(mode, a.co, t, xin[j], e4[j], a.cond ? cin[j] : 0.f, zz);
      }
      if (n4 + 3 < n_end) *(f32x4*)(xrow + n4) = o;
      else
        for (int j = 0; j < 4 && n4 + j < n_end; ++j) xrow[n4 + j] = o[j];
    }
  }
  SDDM_STAMP_AT(a, 6, ftile + b * (F / FT));
  SDDM_STAMP_AT(a, 7, ftile + b * (F / FT));
}

hipError_t launch_final(int dtype, const FinalArgs& a, int B, hipStream_t s) {
  const int back = a.W / a.S - 1, YR = a.FT + back;
  const size_t lds = ((size_t)9 * (YR + 2) * (a.W + 2) + (size_t)YR * a.W + 2 * a.C) * 4;
  // 16-frame tiles as one 16-wave block per CU (less halo re-transform than 8-frame tiles, and
  // the whole grid resident in one round); one pass of 4 samples per thread covers a block's
  // samples (the last block's tail included)
  const int nt = a.FT >= 16 ? 1024 : 512;
  if (lds > kLdsBytes || a.F % a.FT || a.C != 32 || a.FT * a.S + a.W > 4 * nt || a.N % 4) return hipErrorInvalidValue;
  static const bool xcd = !std::getenv("SDDM_FINAL_XCD") || std::atoi(std::getenv("SDDM_FINAL_XCD")) != 0;
  const dim3 grid = xcd ? dim3((a.F / a.FT) * B) : dim3(a.F / a.FT, B);
  static const bool generic = std::getenv("SDDM_NO_FINAL_SHAPES") != nullptr;   // A/B runs
  constexpr FinalShape h = kFinalShapes[1];
  const bool shaped = !generic && dtype != DT_F32 && nt == 512 && a.FT == h.FT && a.W == h.W && a.S == h.S &&
                      a.F == h.F && a.N == h.N && a.C == h.C && a.gtiles == h.GT && a.gntile == h.GNT && a.groups == h.G;
#define SDDM_FINAL(TT)                                                                                      \
  if (shaped && a.mode == 4) hipLaunchKernelGGL((final_kernel<TT, 512, 1, 4>), grid, dim3(512), lds, s, a);   \
  else if (shaped) hipLaunchKernelGGL((final_kernel<TT, 512, 1, kFinalModeArg>), grid, dim3(512), lds, s, a); \
  else if (nt == 1024) hipLaunchKernelGGL((final_kernel<TT, 1024, 0, kFinalModeArg>), grid, dim3(1024), lds, s, a); \
  else hipLaunchKernelGGL((final_kernel<TT, 512, 0, kFinalModeArg>), grid, dim3(512), lds, s, a);
  if (dtype == DT_F32) { SDDM_FINAL(float) }
  else if (dtype == DT_BF16) { SDDM_FINAL(bf16_t) }
  else { SDDM_FINAL(f16_t) }
#undef SDDM_FINAL
  return hipGetLastError();
}

hipError_t launch_transition(const TransArgs& a, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>((a.total + 255) / 256, 4096);
  hipLaunchKernelGGL(transition_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_init_state(const InitArgs& a, hipStream_t s) {
  const int64_t blocks = std::min<int64_t>((a.total + 255) / 256, 4096);
  hipLaunchKernelGGL(init_state_kernel, dim3((unsigned)std::max<int64_t>(blocks, 1)), dim3(256), 0, s, a);
  return hipGetLastError();
}

__global__ void set_int_kernel(int* p, int v) { *p = v; }
__global__ void set_params_kernel(StepParams* p, int t, uint64_t seed, int64_t row_offset) {
  p->t = t; p->seed = seed; p->row_offset = row_offset;
}
hipError_t launch_set_params(StepParams* p, int t, uint64_t seed, int64_t row_offset, hipStream_t s) {
  hipLaunchKernelGGL(set_params_kernel, dim3(1), dim3(1), 0, s, p, t, seed, row_offset);
  return hipGetLastError();
}
// holds a stream for `ticks` of the 100 MHz realtime counter (bounded: at most ~10^6 polls)
__global__ void delay_kernel(unsigned ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 1000000; ++i) {
    if (__builtin_amdgcn_s_memrealtime() - t0 >= ticks) break;
    __builtin_amdgcn_s_sleep(8);
  }
}
hipError_t launch_delay(unsigned us, hipStream_t s) {
  hipLaunchKernelGGL(delay_kernel, dim3(1), dim3(64), 0, s, us * 100u);
  return hipGetLastError();
}
hipError_t launch_set_int(int* p, int v, hipStream_t s) {
  hipLaunchKernelGGL(set_int_kernel, dim3(1), dim3(1), 0, s, p, v);
  return hipGetLastError();
}

}  // namespace sddm
