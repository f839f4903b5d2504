// Whole-K-resident 3x3 convolution for the narrow UNet levels (segment width <= 32: the 64x32 ...
// 8x4 images with 64..320 channels of UNetModified2.py:146-235), every stride-2 Downsample
// (UNetModified2.py:103-109) and the nearest-2x Upsample convs (UNetModified2.py:93-100) landing
// there, and any wide layer whose input does not fit the row-streaming kernel.
//
// These layers are small GEMMs (M = B*pixels = 512..32768, N = Cout = 64..160, K = 9*Cin up to
// 2880 + the 1x1 res_conv) whose cost is latency and instruction issue, not bandwidth.  A block
// (4 waves, two blocks per CU so one block's staging overlaps the other's MFMAs) owns MT output
// pixels of one image x 32 output channels and
//   1. issues, before anything waits: the first weight fragments of every wave, the producer's
//      GroupNorm tile statistics and the raw input halo of all input channels (plus the raw
//      ResnetBlock.res_conv input), every load unconditional (clamped addresses) so the
//      compiler keeps them all in flight;
//   2. finalizes GroupNorm (fp64 Chan combination, fixed order), applies GN + SiLU, resolves the
//      nearest upsample / stride-2 halo / virtual channel concat / zero padding, and writes a
//      plane-major LDS image (a plane = one 16-byte channel unit of every halo pixel; plane
//      stride = 0 mod 256 B so the ds_read_b128 lane groups of an MFMA operand never collide;
//      staging writes go 8 consecutive pixels of one plane per 8-lane group, conflict free);
//   3. splits K (taps x 32-channel chunks, then the res_conv chunks) round-robin over the 4 waves;
//      each wave streams its weight fragments from L2 through a D-deep register ring while the
//      pixel fragments come from LDS;
//   4. reduces the 4 partial tiles through LDS in a fixed order (deterministic), adds bias +
//      noise embedding + identity residual, stores 4-channel vectors, and reduces the GroupNorm
//      statistics of the stored values from registers (shuffles + one LDS exchange).
// If the input does not fit in LDS the chunks are processed in batches (one round trip each).
#include "conv_common.h"
#include "kernels.h"

namespace sddm {

struct DeepGeo { int HR, HC, HP, PLB, PLR; };

__host__ __device__ inline DeepGeo deep_geo(bool s2, int TR, int TW, int MT) {
  DeepGeo d;
  d.HR = s2 ? 2 * TR + 1 : TR + 2;
  d.HC = s2 ? 2 * TW + 1 : TW + 2;
  d.HP = d.HR * d.HC;
  d.PLB = (d.HP * 16 + 255) / 256 * 256;
  d.PLR = (MT * 16 + 255) / 256 * 256;
  return d;
}

// Chan merge of (n, mean, M2) partial statistics
__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  const float nt = n + nb;
  if (nb == 0.f) return;
  if (n == 0.f) { n = nb; mean = meanb; m2 = m2b; return; }
  const float d = meanb - mean;
  mean += d * (nb / nt);
  m2 += m2b + d * d * (n * nb / nt);
  n = nt;
}

template <typename T, bool S2, int MT>
__global__ __launch_bounds__(256, 2) void conv_deep_kernel(ConvArgs a) {
  constexpr int ES = (int)sizeof(T);
  constexpr int UPP = 2 * ES;          // 16-byte planes per 32-channel chunk
  constexpr int UPL = ES / 2;          // planes per MFMA lane group (8 channels)
  constexpr int VE = 16 / ES;          // channels per plane
  constexpr int FP = MT / 16, FC = 2, NB = 32, NBP = NB + 4;
  constexpr int MAXU = 8;              // staged 16-byte units per thread per round trip
  constexpr int D = (ES == 4 ? 4 : 8) / (MT >= 128 ? 2 : 1);   // weight-fragment ring depth
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int tile = blockIdx.x, b = blockIdx.y, n0 = blockIdx.z * NB;
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  const int y0 = ty * a.TR, x0 = tx * a.TW;
  const int npv = a.TR * a.TW;         // valid pixels (< MT only for images smaller than a tile)
  const DeepGeo geo = deep_geo(S2, a.TR, a.TW, MT);
  const int HC = geo.HC, HP = geo.HP, PLB = geo.PLB, PLR = geo.PLR;
  const int Cin = a.CA + a.CB, nck = Cin / 32;
  const int RC = a.RCA + a.RCB, rck = a.res_mode == 2 ? RC / 32 : 0;
  const int CBT = a.ck_batch;
  const bool gn = a.gamma != nullptr;
  const int res_off = CBT * UPP * PLB;
  float* gsc = (float*)(smem + res_off + rck * UPP * PLR);   // [2][Cin]
  const int img_in = a.Hi * a.Wi;
  const T* srcA = (const T*)a.srcA + (size_t)b * img_in * a.CA;
  const T* srcB = a.CB ? (const T*)a.srcB + (size_t)b * img_in * a.CB : srcA;
  const int img_out = a.Ho * a.Wo;
  const T* rawA = a.res_mode == 2 ? (const T*)a.rawA + (size_t)b * img_out * a.RCA : srcA;
  const T* rawB = (a.res_mode == 2 && a.RCB) ? (const T*)a.rawB + (size_t)b * img_out * a.RCB : rawA;
  SDDM_STAMP(a, 0);

  // epilogue constants of this thread's 4 output channels (fixed for the whole block)
  const int ec4 = (tid & 7) * 4;
  float badd[4];
  {
    const int t_now = a.t_dev ? *a.t_dev : 0;
    const float* trow = a.temb ? a.temb + (size_t)(a.temb_per_b ? b : t_now) * a.temb_ld : nullptr;
#pragma unroll
    for (int i = 0; i < 4; ++i) badd[i] = a.bias[n0 + ec4 + i] + (trow ? trow[n0 + ec4 + i] : 0.f);
  }
  GNLoad gl;
  const GNFuse gf{a.gstA, a.gtilesA, a.gntileA, a.gstB, a.gtilesB, a.gntileB, a.gamma, a.beta, a.groups, a.eps};
  if (gn) gl.issue(gf, b, a.CA, a.CB);

  int pix_off[FP];
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    int p = fp * 16 + (lane & 15);
    if (p >= npv) p = 0;
    const int py = p / a.TW, px = p - py * a.TW;
    pix_off[fp] = S2 ? ((2 * py) * HC + 2 * px) * 16 : (py * HC + px) * 16;
  }
  f32x4 acc[FP][FC];
#pragma unroll
  for (int i = 0; i < FP; ++i)
#pragma unroll
    for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const size_t w3 = (size_t)nck * 9 * 32;              // elements per packed 3x3 weight row
  const float rHC = 1.0f / (float)HC, rTW = 1.0f / (float)a.TW;
  const int nbatch = (nck + CBT - 1) / CBT;
  bool gn_pending = gn;
  for (int bi = 0; bi < nbatch; ++bi) {
    const int c_lo = bi * CBT, c_hi = min(nck, c_lo + CBT);
    const bool last = bi == nbatch - 1;
    const int nq3 = (c_hi - c_lo) * UPP;
    const int n3 = (HP + 7) / 8 * 8 * nq3;
    const int nqr = last ? rck * UPP : 0;
    const int total = n3 + nqr * MT;
    const float rnq3 = 1.0f / (float)max(nq3, 1), rnqr = 1.0f / (float)max(nqr, 1);
    // ---- this batch's K steps (wave-uniform, SGPRs) and the first D weight fragments ----
    const int ns3 = (c_hi - c_lo) * 9;
    const int ns = ns3 + nqr / UPP;
    const int nj = (wv < ns && !(a.dbg & 8)) ? (ns - wv + 3) / 4 : 0;
    const int s_last = wv + 4 * max(nj - 1, 0);
    const T* wbase = (const T*)a.wgt + (size_t)(n0 + (lane & 15)) * w3 + (size_t)c_lo * 9 * 32 + g * 8;
    const T* rbase = (const T*)a.res_wgt + (size_t)(n0 + (lane & 15)) * RC + g * 8;
    auto wfrag = [&](int s, int fc) -> Frag<T> {
      if (s < ns3) return load_frag<T>((const char*)(wbase + (size_t)fc * 16 * w3 + (size_t)s * 32));
      return load_frag<T>((const char*)(rbase + (size_t)fc * 16 * RC + (s - ns3) * 32));
    };
    Frag<T> wa[D][FC];
    if (nj > 0) {
#pragma unroll
      for (int d = 0; d < D; ++d)
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) wa[d][fc] = wfrag(min(wv + 4 * d, s_last), fc);
    }
    if (bi > 0) __syncthreads();                       // previous batch's readers are done
    // ---------------- staging: global -> registers -> (GN + SiLU) -> LDS ----------------
    for (int u0 = 0; u0 < total; u0 += MAXU * 256) {
      f32x4 reg[MAXU];
      int dst[MAXU], gsel[MAXU];
#pragma unroll
      for (int k = 0; k < MAXU; ++k) {
        const int u = u0 + tid + k * 256;
        const T* ptr = srcA;                           // any valid address; result unused if dst < 0
        int d = -1, gs = -1;
        if (u < n3) {                                  // 8 lanes = 8 consecutive halo pixels of one plane
          const int grp = u >> 3, gq = fdivi(grp, rnq3), q = grp - gq * nq3, hp = gq * 8 + (u & 7);
          const int hy = fdivi(hp, rHC), hx = hp - hy * HC;
          int iy, ix;
          bool ok;
          if (S2) {
            iy = 2 * y0 - 1 + hy; ix = 2 * x0 - 1 + hx;
            ok = iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi;
          } else {
            iy = y0 - 1 + hy; ix = x0 - 1 + hx;
            ok = iy >= 0 && iy < a.Ho && ix >= 0 && ix < a.Wo;
            if (a.upsample) { iy >>= 1; ix >>= 1; }
          }
          const int c = c_lo * 32 + q * VE;
          const bool fromA = c < a.CA;
          if (ok) ptr = (fromA ? srcA : srcB) + (iy * a.Wi + ix) * (fromA ? a.CA : a.CB) + (fromA ? c : c - a.CA);
          if (hp < HP) { d = q * PLB + hp * 16; gs = ok ? c : -2; }
        } else if (u < total) {                        // raw res_conv input at the output pixels
          const int v = u - n3, grp = v >> 3, gq = fdivi(grp, rnqr), q = grp - gq * nqr, p = gq * 8 + (v & 7);
          d = res_off + q * PLR + p * 16;
          gs = -2;
          if (p < npv) {
            const int py = fdivi(p, rTW), px = p - py * a.TW;
            const int c = q * VE;
            const bool fromA = c < a.RCA;
            ptr = (fromA ? rawA : rawB) + ((y0 + py) * a.Wo + (x0 + px)) * (fromA ? a.RCA : a.RCB) +
                  (fromA ? c : c - a.RCA);
            gs = -1;
          }
        }
        reg[k] = *(const f32x4*)ptr;
        dst[k] = d;
        gsel[k] = gs;
      }
      SDDM_STAMP(a, 1);
      if (gn_pending) {
        gl.finish(gf, b, a.CA, a.CB, gsc, gsc + Cin);
        gn_pending = false;
        __syncthreads();                               // scale / shift visible
      }
      SDDM_STAMP(a, 2);
#pragma unroll
      for (int k = 0; k < MAXU; ++k) {
        if (dst[k] < 0) continue;
        f32x4 v = reg[k];
        if (gsel[k] == -2) v = f32x4{0.f, 0.f, 0.f, 0.f};                 // zero padding
        else if (gn && gsel[k] >= 0) v = transform_lds<T>(v, gsc + gsel[k], gsc + Cin + gsel[k]);
        *(f32x4*)(smem + dst[k]) = v;
      }
    }
    __syncthreads();
    SDDM_STAMP(a, 3);
    // ---------------- this wave's K steps: round-robin over the 4 waves ----------------
    // every ring refill is unconditional (clamped to the wave's last step) so the compiler's
    // vmcnt accounting keeps D fragment loads in flight
    for (int j0 = 0; j0 < nj; j0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int j = j0 + d;
        const int s = wv + 4 * j;
        if (j < nj) {
          Frag<T> bf[FP];
          if (s < ns3) {
            const int lc = s / 9, tap = s - 9 * lc, dy = tap / 3, dx = tap - 3 * dy;
            const char* pb = smem + (lc * UPP + g * UPL) * PLB + (dy * HC + dx) * 16;
#pragma unroll
            for (int fp = 0; fp < FP; ++fp) bf[fp] = load_planes<T>(pb + pix_off[fp], PLB);
          } else {
            const char* pb = smem + res_off + ((s - ns3) * UPP + g * UPL) * PLR + (lane & 15) * 16;
#pragma unroll
            for (int fp = 0; fp < FP; ++fp) bf[fp] = load_planes<T>(pb + fp * 256, PLR);
          }
#pragma unroll
          for (int fc = 0; fc < FC; ++fc)
#pragma unroll
            for (int fp = 0; fp < FP; ++fp) mfma_frag(acc[fp][fc], wa[d][fc], bf[fp]);
        }
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) wa[d][fc] = wfrag(min(s + 4 * D, s_last), fc);
      }
    }
  }
  // identity residual of this thread's output pixels: issued before the reduction barrier
  constexpr int PPI = 256 / (NB / 4);                 // pixels per epilogue pass (32)
  constexpr int EIT = (MT + PPI - 1) / PPI;
  typedef T vec4 __attribute__((ext_vector_type(4)));
  vec4 rres[EIT];
  if (a.res_mode == 1) {
    const T* rs = (const T*)a.res_src + (size_t)b * img_out * a.Cout + n0 + ec4;
#pragma unroll
    for (int it = 0; it < EIT; ++it) {
      int p = it * PPI + (tid >> 3);
      if (p >= npv) p = 0;
      const int py = fdivi(p, rTW), px = p - py * a.TW;
      rres[it] = *(const vec4*)(rs + ((y0 + py) * a.Wo + (x0 + px)) * a.Cout);
    }
  }
  SDDM_STAMP(a, 4);
  __syncthreads();
  // ---------------- reduce the 4 partial tiles: red[wave][MT][NBP] ----------------
  float* red = (float*)smem;
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    const int p = fp * 16 + (lane & 15);
#pragma unroll
    for (int fc = 0; fc < FC; ++fc) *(f32x4*)(red + (wave * MT + p) * NBP + fc * 16 + 4 * g) = acc[fp][fc];
  }
  __syncthreads();
  float sn = 0.f, sk[4], s1[4], s2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { sk[i] = 0.f; s1[i] = 0.f; s2[i] = 0.f; }
  T* out = (T*)a.out + (size_t)b * img_out * a.Cout + n0 + ec4;
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int p = it * PPI + (tid >> 3);
    if (p < npv) {
      const int py = fdivi(p, rTW), px = p - py * a.TW;
      f32x4 s = *(const f32x4*)(red + p * NBP + ec4);
#pragma unroll
      for (int w = 1; w < 4; ++w) s += *(const f32x4*)(red + (w * MT + p) * NBP + ec4);
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = s[i] + badd[i];
      if (a.res_mode == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += (float)rres[it][i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = round_t<T>(v[i]);
      store4<T>(out + ((y0 + py) * a.Wo + (x0 + px)) * a.Cout, v[0], v[1], v[2], v[3]);
      if (it == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) sk[i] = v[i];     // shift = first value (stable sums)
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float dlt = v[i] - sk[i];
        s1[i] += dlt;
        s2[i] += dlt * dlt;
      }
      sn += 1.f;
    }
  }
  SDDM_STAMP(a, 5);
  if (a.stats) {
    // per-thread (n, mean, M2) -> lanes of one channel group (xor 8, 16, 32) -> 4 waves via LDS;
    // full tiles give every thread the same count, so the merges need no division
    const bool even = (npv & (PPI - 1)) == 0;
    float mn[4], m2[4], nn = sn;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float inv = sn > 0.f ? 1.0f / sn : 0.f;
      mn[i] = sk[i] + s1[i] * inv;
      m2[i] = fmaxf(s2[i] - s1[i] * s1[i] * inv, 0.f);
    }
    if (even) {
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float mb = __shfl_xor(mn[i], o), qb = __shfl_xor(m2[i], o);
          const float d = mb - mn[i];
          m2[i] += qb + d * d * (nn * 0.5f);
          mn[i] += 0.5f * d;
        }
        nn *= 2.f;
      }
    } else {
      float nv[4] = {nn, nn, nn, nn};
#pragma unroll
      for (int o = 8; o < 64; o <<= 1)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float nb = __shfl_xor(nv[i], o), mb = __shfl_xor(mn[i], o), qb = __shfl_xor(m2[i], o);
          chan_merge(nv[i], mn[i], m2[i], nb, mb, qb);
        }
      nn = nv[0];
    }
    __syncthreads();                                   // red reads done
    float* xs = red;                                   // [4 waves][8 groups][4 ch][3]
    if (lane < 8)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float* e = xs + ((wave * 8 + lane) * 4 + i) * 3;
        e[0] = nn; e[1] = mn[i]; e[2] = m2[i];
      }
    __syncthreads();
    if (tid < NB) {
      const int grp = tid >> 2, i = tid & 3;
      float n = 0.f, mean = 0.f, q = 0.f;
      for (int w = 0; w < 4; ++w) {
        const float* e = xs + ((w * 8 + grp) * 4 + i) * 3;
        chan_merge(n, mean, q, e[0], e[1], e[2]);
      }
      float* dst = a.stats + (((size_t)b * a.n_tiles + tile) * a.Cout + n0 + tid) * 2;
      dst[0] = mean * n;
      dst[1] = q;
    }
  }
  SDDM_STAMP(a, 6);
  SDDM_STAMP(a, 7);
}

template <typename T, bool S2, int MT>
static size_t deep_lds(const ConvArgs& a, int ck_batch) {
  constexpr int ES = (int)sizeof(T), UPP = 2 * ES;
  const DeepGeo geo = deep_geo(S2, a.TR, a.TW, MT);
  const int Cin = a.CA + a.CB, rck = a.res_mode == 2 ? (a.RCA + a.RCB) / 32 : 0;
  const size_t stage = (size_t)ck_batch * UPP * geo.PLB + (size_t)rck * UPP * geo.PLR + (size_t)2 * Cin * 4;
  const size_t red = (size_t)4 * MT * (32 + 4) * 4;
  return stage > red ? stage : red;
}

template <typename T, bool S2, int MT>
static hipError_t deep_go(const ConvArgs& a, int B, hipStream_t s, size_t* lo) {
  if (lo) {
    *lo = deep_lds<T, S2, MT>(a, a.ck_batch);
    return hipSuccess;
  }
  const int nck = (a.CA + a.CB) / 32;
  if (a.ck_batch < 1 || a.ck_batch > nck || a.TR * a.TW > MT || a.Cout % 32 || (a.CA + a.CB) % 32)
    return hipErrorInvalidValue;
  const size_t lds = deep_lds<T, S2, MT>(a, a.ck_batch);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL((conv_deep_kernel<T, S2, MT>), dim3(a.n_tiles, B, a.Cout / 32), dim3(256), lds, s, a);
  return hipGetLastError();
}

template <typename T>
static hipError_t deep_dispatch(int mt, bool s2, const ConvArgs& a, int B, hipStream_t s, size_t* lo) {
#define SDDM_DEEP(S2V, MTV) \
  if (s2 == S2V && mt == MTV) return deep_go<T, S2V, MTV>(a, B, s, lo);
  SDDM_DEEP(false, 32) SDDM_DEEP(false, 64) SDDM_DEEP(false, 128)
  SDDM_DEEP(true, 32) SDDM_DEEP(true, 64) SDDM_DEEP(true, 128)
#undef SDDM_DEEP
  if (lo) *lo = (size_t)1 << 40;
  return hipErrorInvalidValue;
}

hipError_t launch_conv_deep(int dtype, int mt, bool s2, const ConvArgs& a, int B, hipStream_t s) {
  if (dtype == DT_F32) return deep_dispatch<float>(mt, s2, a, B, s, nullptr);
  if (dtype == DT_BF16) return deep_dispatch<bf16_t>(mt, s2, a, B, s, nullptr);
  return deep_dispatch<f16_t>(mt, s2, a, B, s, nullptr);
}

size_t conv_deep_lds_bytes(int dtype, int mt, bool s2, const ConvArgs& a) {
  size_t lo = (size_t)1 << 40;
  if (dtype == DT_F32) (void)deep_dispatch<float>(mt, s2, a, 1, 0, &lo);
  else if (dtype == DT_BF16) (void)deep_dispatch<bf16_t>(mt, s2, a, 1, 0, &lo);
  else (void)deep_dispatch<f16_t>(mt, s2, a, 1, 0, &lo);
  return lo;
}

}  // namespace sddm
