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
#include <algorithm>

namespace sddm {

static __device__ __forceinline__ int round16(int x) { return (x + 15) & ~15; }

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
// Per-channel tile statistics from an fp32 LDS tile [npix][ld] (values already rounded to the
// storage type).  Writes (sum, M2 about the tile mean) for channels [0, nch).
// =============================================================================================
__device__ void tile_channel_stats(const float* tile, int ld, int npix, int nch, float* dst,
                                   int dst_stride) {
  // threads split as (channel, part); parts combine through shuffles within a wave group
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int parts = max(1, min(nthr / max(nch, 1), 16));
  // round parts down to power of two
  int p2 = 1;
  while (p2 * 2 <= parts) p2 *= 2;
  const int c = tid / p2, part = tid % p2;
  float s = 0.f;
  const bool act = c < nch;
  if (act)
    for (int p = part; p < npix; p += p2) s += tile[p * ld + c];
  for (int o = 1; o < p2; o <<= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)npix;
  float m2 = 0.f;
  if (act)
    for (int p = part; p < npix; p += p2) {
      const float d = tile[p * ld + c] - mean;
      m2 += d * d;
    }
  for (int o = 1; o < p2; o <<= 1) m2 += __shfl_xor(m2, o);
  if (act && part == 0) {
    dst[c * dst_stride] = s;
    dst[c * dst_stride + 1] = m2;
  }
}

// =============================================================================================
// conv_in: SignalToFrames on cond and x_t (idx[f,w] = S*f + w), channel concat, Conv2d(2, C, 3,
// pad 1) + bias.  One thread per output pixel, TR frame rows per block.
// =============================================================================================
template <typename T>
__global__ __launch_bounds__(256) void conv_in_kernel(ConvInArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* wl = (float*)smem;                 // [Cout][2][9] + bias
  float* otile = wl + a.Cout * 18 + a.Cout; // [TR*W][Cout+1]
  const int b = blockIdx.y, f0 = blockIdx.x * a.TR, tid = threadIdx.x;
  if (a.t_dev && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0) *a.t_dev -= 1;
  for (int i = tid; i < a.Cout * 18; i += blockDim.x) wl[i] = a.w[i];
  for (int i = tid; i < a.Cout; i += blockDim.x) wl[a.Cout * 18 + i] = a.bias[i];
  __syncthreads();
  const int ld = a.Cout + 1, npix = a.TR * a.W;
  const float* cnd = a.cond + (size_t)b * a.N;
  const float* xx = a.x + (size_t)b * a.N;
  for (int p = tid; p < npix; p += blockDim.x) {
    const int f = f0 + p / a.W, w = p % a.W;
    float in0[9], in1[9];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const int ff = f + dy - 1, ww = w + dx - 1;
        const bool ok = ff >= 0 && ff < a.F && ww >= 0 && ww < a.W;
        const int n = ff * a.S + ww;
        in0[dy * 3 + dx] = ok ? cnd[n] : 0.f;
        in1[dy * 3 + dx] = ok ? xx[n] : 0.f;
      }
    for (int co = 0; co < a.Cout; ++co) {
      const float* wc = wl + co * 18;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) s += wc[k] * in0[k];
#pragma unroll
      for (int k = 0; k < 9; ++k) s += wc[9 + k] * in1[k];
      s += wl[a.Cout * 18 + co];
      otile[p * ld + co] = to_f32<T>(from_f32<T>(s));
    }
  }
  __syncthreads();
  // store NHWC rows (contiguous: TR*W pixels * Cout channels)
  T* out = (T*)a.out + ((size_t)b * a.F + f0) * a.W * a.Cout;
  for (int i = tid; i < npix * a.Cout; i += blockDim.x) out[i] = from_f32<T>(otile[(i / a.Cout) * ld + i % a.Cout]);
  tile_channel_stats(otile, ld, npix, a.Cout,
                     a.stats + ((size_t)b * (a.F / a.TR) + blockIdx.x) * a.Cout * 2, 2);
}

hipError_t launch_conv_in(int dtype, const ConvInArgs& a, int B, hipStream_t s) {
  const size_t lds = (size_t)(a.Cout * 19) * 4 + (size_t)a.TR * a.W * (a.Cout + 1) * 4;
  dim3 grid(a.F / a.TR, B);
  if (dtype == DT_F32) hipLaunchKernelGGL(conv_in_kernel<float>, grid, dim3(256), lds, s, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(conv_in_kernel<bf16_t>, grid, dim3(256), lds, s, a);
  else hipLaunchKernelGGL(conv_in_kernel<f16_t>, grid, dim3(256), lds, s, a);
  return hipGetLastError();
}

// =============================================================================================
// MFMA implicit-GEMM 3x3 convolution.
//   D[co][pixel] = sum_{tap, ci} W[co][tap][ci] * X[pixel + tap][ci]
// A operand = weights (rows = output channels), B operand = input pixels (cols), so each lane's
// accumulator holds 4 consecutive channels of one pixel (C/D layout: col = lane & 15,
// row = 4 * (lane >> 4) + i).  The K loop walks 32-channel chunks; per chunk the block stages
// the transformed halo tile and the weight slab in LDS.
// Block = 4 waves stacked along pixels; wave tile = (FP*16 pixels) x (FC*16 channels).
// =============================================================================================
template <typename T> struct Mfma;
template <> struct Mfma<bf16_t> {
  typedef bf16x8 frag;
  static __device__ __forceinline__ void run(f32x4& acc, const char* pa, const char* pb) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(const bf16x8*)pa, *(const bf16x8*)pb, acc, 0, 0, 0);
  }
};
template <> struct Mfma<f16_t> {
  static __device__ __forceinline__ void run(f32x4& acc, const char* pa, const char* pb) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(*(const f16x8*)pa, *(const f16x8*)pb, acc, 0, 0, 0);
  }
};
template <> struct Mfma<float> {
  // 8 channels per lane group: MFMA j consumes element j (k-set {j, 8+j, 16+j, 24+j}).
  static __device__ __forceinline__ void run(f32x4& acc, const char* pa, const char* pb) {
    const f32x4 a0 = *(const f32x4*)pa, a1 = *(const f32x4*)(pa + 16);
    const f32x4 b0 = *(const f32x4*)pb, b1 = *(const f32x4*)(pb + 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j], b0[j], acc, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j], b1[j], acc, 0, 0, 0);
  }
};

template <typename T>
__device__ __forceinline__ void transform16(char* dst, const char* src, const float* sc, const float* sh,
                                            bool gn) {
  // 16 bytes = 16/sizeof(T) elements; GN affine + SiLU in fp32, re-round to T
  constexpr int VE = 16 / (int)sizeof(T);
  typedef T vec __attribute__((ext_vector_type(VE)));
  vec v = *(const vec*)src;
  if (gn) {
#pragma unroll
    for (int j = 0; j < VE; ++j) v[j] = from_f32<T>(silu(to_f32<T>(v[j]) * sc[j] + sh[j]));
  }
  *(vec*)dst = v;
}

template <int ES> struct LdsGeom {
  static constexpr int CK = 32;
  static constexpr int PIX = CK * ES + 16;       // bytes per halo pixel (16-B pad vs bank conflicts)
  static constexpr int WROW = 9 * CK * ES + 16;  // bytes per output channel of a weight chunk
  static constexpr int RROW = CK * ES + 16;      // bytes per output channel of a 1x1 chunk
};

template <typename T, bool S2, int FP, int FC>
__global__ __launch_bounds__(256) void conv3x3_kernel(ConvArgs a) {
  constexpr int WM = 4;
  constexpr int ES = (int)sizeof(T);
  typedef LdsGeom<ES> G;
  constexpr int CK = G::CK, PIX = G::PIX, WROW = G::WROW, RROW = G::RROW;
  constexpr int MBLK = WM * FP * 16, NBLK = FC * 16;
  constexpr int UPP = CK * ES / 16;  // 16-byte units per pixel chunk
  constexpr int VE = 16 / ES;
  constexpr int LG = 8 * ES;         // bytes of one lane group's 8 channels
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tile = blockIdx.x, b = blockIdx.y, n0 = blockIdx.z * NBLK;
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  const int y0 = ty * a.TR, x0 = tx * a.TW;
  const int HR = S2 ? 2 * a.TR + 1 : a.TR + 2, HC = S2 ? 2 * a.TW + 1 : a.TW + 2;
  const int Cin = a.CA + a.CB;
  const bool gn = a.gn_scale != nullptr;
  const bool res2 = a.res_mode == 2;

  char* halo = smem;
  char* wl = halo + round16(HR * HC * PIX);
  char* raw = wl + NBLK * WROW;
  char* rw = raw + (res2 ? MBLK * PIX : 0);
  float* gsc = (float*)(rw + (res2 ? NBLK * RROW : 0));

  const int npix_valid = a.TR * a.TW;
  int pix_off[FP];
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    int p = wave * FP * 16 + fp * 16 + (lane & 15);
    if (p >= npix_valid) p = 0;
    const int py = p / a.TW, px = p - py * a.TW;
    pix_off[fp] = ((S2 ? 2 * py : py) * HC + (S2 ? 2 * px : px)) * PIX + (lane >> 4) * LG;
  }
  f32x4 acc[FP][FC];
#pragma unroll
  for (int i = 0; i < FP; ++i)
#pragma unroll
    for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const size_t img_in = (size_t)a.Hi * a.Wi;
  const int nchunk = Cin / CK;
  for (int ck = 0; ck < nchunk; ++ck) {
    const int c0 = ck * CK;
    const bool fromA = c0 < a.CA;
    const T* src = fromA ? (const T*)a.srcA : (const T*)a.srcB;
    const int Cs = fromA ? a.CA : a.CB;
    const int cs0 = fromA ? c0 : c0 - a.CA;
    __syncthreads();
    if (gn && tid < CK) {
      gsc[tid] = a.gn_scale[(size_t)b * Cin + c0 + tid];
      gsc[CK + tid] = a.gn_shift[(size_t)b * Cin + c0 + tid];
    }
    // weight slab: rows n0..n0+NBLK, chunk ck, 9 taps x 32 channels (contiguous per row)
    for (int u = tid; u < NBLK * 9 * UPP; u += 256) {
      const int row = u / (9 * UPP), q = u - row * 9 * UPP;
      const char* g = (const char*)a.wgt + (((size_t)(n0 + row) * nchunk + ck) * 9 * CK) * ES + q * 16;
      *(f32x4*)(wl + row * WROW + q * 16) = *(const f32x4*)g;
    }
    if (gn) __syncthreads();  // gsc visible to the halo transform
    for (int u = tid; u < HR * HC * UPP; u += 256) {
      const int hp = u / UPP, q = u - hp * UPP;
      const int hy = hp / HC, hx = hp - hy * HC;
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
      char* dst = halo + hp * PIX + q * 16;
      if (ok) {
        const size_t pi = (size_t)b * img_in + (size_t)iy * a.Wi + ix;
        transform16<T>(dst, (const char*)(src + pi * Cs + cs0) + q * 16, gsc + q * VE, gsc + CK + q * VE, gn);
      } else {
        *(f32x4*)dst = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    __syncthreads();
    const char* wbase = wl + (lane & 15) * WROW + (lane >> 4) * LG;
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap - dy * 3;
      const int toff = (dy * HC + dx) * PIX;
#pragma unroll
      for (int fc = 0; fc < FC; ++fc)
#pragma unroll
        for (int fp = 0; fp < FP; ++fp)
          Mfma<T>::run(acc[fp][fc], wbase + fc * 16 * WROW + tap * CK * ES, halo + pix_off[fp] + toff);
    }
  }
  // ---- fused ResnetBlock.res_conv: 1x1 over the raw block input (K = RCA + RCB) ----
  if (res2) {
    const int rcin = a.RCA + a.RCB;
    for (int c0 = 0; c0 < rcin; c0 += CK) {
      const bool fromA = c0 < a.RCA;
      const T* src = fromA ? (const T*)a.rawA : (const T*)a.rawB;
      const int Cs = fromA ? a.RCA : a.RCB;
      const int cs0 = fromA ? c0 : c0 - a.RCA;
      __syncthreads();
      for (int u = tid; u < NBLK * UPP; u += 256) {
        const int row = u / UPP, q = u - row * UPP;
        const char* g = (const char*)a.res_wgt + ((size_t)(n0 + row) * rcin + c0) * ES + q * 16;
        *(f32x4*)(rw + row * RROW + q * 16) = *(const f32x4*)g;
      }
      for (int u = tid; u < MBLK * UPP; u += 256) {
        const int p = u / UPP, q = u - p * UPP;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (p < npix_valid) {
          const int py = p / a.TW, px = p - py * a.TW;
          const size_t pi = ((size_t)b * a.Ho + (y0 + py)) * a.Wo + (x0 + px);
          v = *(const f32x4*)((const char*)(src + pi * Cs + cs0) + q * 16);
        }
        *(f32x4*)(raw + p * PIX + q * 16) = v;
      }
      __syncthreads();
      const char* rbase = rw + (lane & 15) * RROW + (lane >> 4) * LG;
#pragma unroll
      for (int fc = 0; fc < FC; ++fc)
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) {
          const int p = wave * FP * 16 + fp * 16 + (lane & 15);
          Mfma<T>::run(acc[fp][fc], rbase + fc * 16 * RROW, raw + p * PIX + (lane >> 4) * LG);
        }
    }
  }
  __syncthreads();
  // ---- epilogue: bias + embedding + residual, round to T, stage in LDS ----
  constexpr int OLD = NBLK + 1;
  float* ot = (float*)smem;
  const int t = a.t_dev ? *a.t_dev : 0;
  const float* trow = a.temb ? a.temb + (size_t)(a.temb_per_b ? b : t) * a.temb_ld : nullptr;
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    const int p = wave * FP * 16 + fp * 16 + (lane & 15);
    const bool pv = p < npix_valid;
    const int py = p / a.TW, px = p - py * a.TW;
    const size_t po = ((size_t)b * a.Ho + (y0 + py)) * a.Wo + (x0 + px);
#pragma unroll
    for (int fc = 0; fc < FC; ++fc) {
      const int cl = fc * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = n0 + cl + i;
        float v = acc[fp][fc][i];
        if (co < a.Cout) {
          v += a.bias[co];
          if (trow) v += trow[co];
          if (a.res_mode == 1 && pv) v += to_f32<T>(((const T*)a.res_src)[po * a.Cout + co]);
        }
        ot[p * OLD + cl + i] = to_f32<T>(from_f32<T>(v));
      }
    }
  }
  __syncthreads();
  // ---- store: each valid pixel writes its NBLK (<= Cout - n0) channels ----
  const int nco = min(NBLK, a.Cout - n0);
  for (int u = tid; u < npix_valid * nco; u += 256) {
    const int p = u / nco, c = u - p * nco;
    const int py = p / a.TW, px = p - py * a.TW;
    const size_t po = ((size_t)b * a.Ho + (y0 + py)) * a.Wo + (x0 + px);
    ((T*)a.out)[po * a.Cout + n0 + c] = from_f32<T>(ot[p * OLD + c]);
  }
  if (a.stats)
    tile_channel_stats(ot, OLD, npix_valid, nco,
                       a.stats + (((size_t)b * a.n_tiles + tile) * a.Cout + n0) * 2, 2);
}

template <typename T, bool S2, int FP, int FC>
static size_t lds_bytes_t(const ConvArgs& a) {
  typedef LdsGeom<(int)sizeof(T)> G;
  constexpr int MBLK = 4 * FP * 16, NBLK = FC * 16;
  const int HR = S2 ? 2 * a.TR + 1 : a.TR + 2, HC = S2 ? 2 * a.TW + 1 : a.TW + 2;
  size_t main = ((size_t)HR * HC * G::PIX + 15) / 16 * 16 + (size_t)NBLK * G::WROW;
  if (a.res_mode == 2) main += (size_t)MBLK * G::PIX + (size_t)NBLK * G::RROW;
  main += 2 * G::CK * 4;
  const size_t epi = (size_t)MBLK * (NBLK + 1) * 4;
  return main > epi ? main : epi;
}

template <typename T, bool S2, int FP, int FC>
static hipError_t launch_t(const ConvArgs& a, int B, hipStream_t s, size_t* lds_only) {
  const size_t lds = lds_bytes_t<T, S2, FP, FC>(a);
  if (lds_only) { *lds_only = lds; return hipSuccess; }
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int nz = (a.Cout + FC * 16 - 1) / (FC * 16);
  hipLaunchKernelGGL((conv3x3_kernel<T, S2, FP, FC>), dim3(a.n_tiles, B, nz), dim3(256), lds, s, a);
  return hipGetLastError();
}

template <typename T>
static hipError_t dispatch_t(const ConvCfg& c, const ConvArgs& a, int B, hipStream_t s, size_t* lo) {
#define SDDM_CONV_CASE(S2V, FPV, FCV)                                                           \
  if (c.stride2 == S2V && c.mblk == 64 * FPV && c.nblk == 16 * FCV)                             \
    return launch_t<T, S2V, FPV, FCV>(a, B, s, lo);
  SDDM_CONV_CASE(0, 1, 2) SDDM_CONV_CASE(0, 2, 2) SDDM_CONV_CASE(0, 1, 4) SDDM_CONV_CASE(0, 2, 4)
  SDDM_CONV_CASE(1, 1, 2) SDDM_CONV_CASE(1, 2, 2) SDDM_CONV_CASE(1, 1, 4) SDDM_CONV_CASE(1, 2, 4)
#undef SDDM_CONV_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_conv3x3(int dtype, const ConvCfg& cfg, const ConvArgs& a, int B, hipStream_t s) {
  if (dtype == DT_F32) return dispatch_t<float>(cfg, a, B, s, nullptr);
  if (dtype == DT_BF16) return dispatch_t<bf16_t>(cfg, a, B, s, nullptr);
  return dispatch_t<f16_t>(cfg, a, B, s, nullptr);
}

size_t conv3x3_lds_bytes(int dtype, const ConvCfg& cfg, const ConvArgs& a) {
  size_t lo = 0;
  if (dtype == DT_F32) (void)dispatch_t<float>(cfg, a, 1, 0, &lo);
  else if (dtype == DT_BF16) (void)dispatch_t<bf16_t>(cfg, a, 1, 0, &lo);
  else (void)dispatch_t<f16_t>(cfg, a, 1, 0, &lo);
  return lo;
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
    const float z = t > 1 ? philox_normal1(a.seed, (uint32_t)t, e) : 0.f;
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
      const float z = philox_normal1(a.seed, 0u, e);
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
// [f0, f0+FT) and the samples [S*f0, S*(f0+FT)) (the last block also the tail up to N); it
// recomputes the W/S-1 preceding frames it needs for the overlap-add.
// =============================================================================================
template <typename T>
__global__ __launch_bounds__(256) void final_kernel(FinalArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.y, f0 = blockIdx.x * a.FT, tid = threadIdx.x;
  const int C = a.C, W = a.W, S = a.S, F = a.F;
  const int back = W / S - 1;                 // extra frames before f0 needed by the OLA
  const int YR = a.FT + back;                 // y rows: frames [f0-back, f0+FT)
  const int IR = YR + 2, IC = W + 2;          // transformed input rows/cols
  const int CL = C + 4;                       // padded channel stride (floats)
  float* in = (float*)smem;                   // [IR][IC][CL]
  float* wl = in + IR * IC * CL;              // [9][C]
  float* y = wl + 9 * C;                      // [YR][W]
  float* gs = y + YR * W;                     // [2][C]
  for (int i = tid; i < C; i += blockDim.x) {
    gs[i] = a.gn_scale[(size_t)b * C + i];
    gs[C + i] = a.gn_shift[(size_t)b * C + i];
  }
  for (int i = tid; i < 9 * C; i += blockDim.x) {
    const int tap = i / C, c = i - tap * C;
    wl[i] = a.w[c * 9 + tap];
  }
  __syncthreads();
  const T* src = (const T*)a.src + (size_t)b * F * W * C;
  for (int u = tid; u < IR * IC * C; u += blockDim.x) {
    const int c = u % C, pp = u / C, ix = pp % IC, iy = pp / IC;
    const int f = f0 - back - 1 + iy, w = ix - 1;
    float v = 0.f;
    if (f >= 0 && f < F && w >= 0 && w < W)
      v = silu(to_f32<T>(src[((size_t)f * W + w) * C + c]) * gs[c] + gs[C + c]);
    in[(iy * IC + ix) * CL + c] = v;
  }
  __syncthreads();
  for (int p = tid; p < YR * W; p += blockDim.x) {
    const int r = p / W, w = p - r * W;
    float s = 0.f;
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap - dy * 3;
      const float* ip = in + ((r + dy) * IC + (w + dx)) * CL;
      const float* wp = wl + tap * C;
      for (int c = 0; c < C; c += 4) {
        const f32x4 v = *(const f32x4*)(ip + c);
        s += wp[c] * v[0] + wp[c + 1] * v[1] + wp[c + 2] * v[2] + wp[c + 3] * v[3];
      }
    }
    y[p] = s + a.bias;
  }
  __syncthreads();
  const int n_begin = f0 * S;
  const int n_end = (f0 + a.FT >= F) ? a.N : (f0 + a.FT) * S;
  const int t = a.t_dev ? *a.t_dev : 0;
  float* xrow = a.x + (size_t)b * a.N;
  const float* crow = a.cond ? a.cond + (size_t)b * a.N : nullptr;
  for (int n = n_begin + tid; n < n_end; n += blockDim.x) {
    // overlapAdd (UNetModified2.py:37-39): frames in ascending order
    int flo = (n - W + S) / S;  // ceil((n - W + 1) / S) for n >= W-1
    if (n - W + 1 <= 0) flo = 0;
    const int fhi = min(F - 1, n / S);
    float e = 0.f;
    for (int f = flo; f <= fhi; ++f) e += y[(f - (f0 - back)) * W + (n - f * S)];
    if (a.mode < 0) {
      a.eps_out[(size_t)b * a.N + n] = e;
    } else {
      const uint64_t ge = (uint64_t)((a.row_offset + b) * (int64_t)a.N + n);
      const float z = t > 1 ? philox_normal1(a.seed, (uint32_t)t, ge) : 0.f;
      xrow[n] = transition_one(a.mode, a.co, t, xrow[n], e, crow ? crow[n] : 0.f, z);
    }
  }
}

hipError_t launch_final(int dtype, const FinalArgs& a, int B, hipStream_t s) {
  const int back = a.W / a.S - 1, YR = a.FT + back;
  const size_t lds = ((size_t)(YR + 2) * (a.W + 2) * (a.C + 4) + 9 * a.C + YR * a.W + 2 * a.C) * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  dim3 grid(a.F / a.FT, B);
  if (dtype == DT_F32) hipLaunchKernelGGL(final_kernel<float>, grid, dim3(256), lds, s, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(final_kernel<bf16_t>, grid, dim3(256), lds, s, a);
  else hipLaunchKernelGGL(final_kernel<f16_t>, grid, dim3(256), lds, s, a);
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
hipError_t launch_set_int(int* p, int v, hipStream_t s) {
  hipLaunchKernelGGL(set_int_kernel, dim3(1), dim3(1), 0, s, p, v);
  return hipGetLastError();
}

}  // namespace sddm
