// DiffWave denoiser (reference model/diffwave.py) for SDDM_spectrogram.infer (model.py:212-257).
//
// Activations are sample-major [B][N][C] in the compute dtype T, so one sample's channels are
// contiguous 16-byte units and every MFMA operand fragment is one vector load.  Per sampling
// call the step-invariant work runs once: the SpectrogramUpsampler (2 ConvTranspose2d passes,
// diffwave.py:48-61) and the conditioner projections of all residual layers
// (conditioner_projection, diffwave.py:93), kept layer-major as cond[L][B][N][2C]; the noise-step
// embedding MLP and every layer's diffusion_projection are tabulated for all t (one row per t).
// Per reverse step: input projection, one fused kernel per residual layer, one output kernel.
//
// Fused residual layer (diffwave.py:90-108), one block = 128 samples of one clip, 4 waves:
//   1. stage y = x + diffusion_projection at the 3 dilated taps (n - d, n, n + d; zero outside
//      the clip: Conv1d zero padding applies to y) into a plane-major LDS image;
//   2. dilated_conv as an MFMA GEMM (K = 3 x 64): wave w owns gate rows [16w, 16w+16) and the
//      matching filter rows [64+16w, ...), so sigmoid(gate) * tanh(filter) pairs sit in the same
//      lane; + bias + conditioner;
//   3. the gated activation goes back to LDS (plane-major) and output_residual / output_projection
//      run as one K = 64 GEMM; the epilogue writes (x + residual) / sqrt(2) to the other x buffer
//      and accumulates the skip sum in fp32.
#include <cstdlib>

#include "conv_common.h"
#include "kernels.h"

namespace sddm {

constexpr int DW_C = 64;            // residual_channels (the kernels are built for 64)
constexpr int DW_MS = 128;          // samples per layer block

__device__ __forceinline__ float dw_silu(float x) { return x * (1.0f / (1.0f + expf(-x))); }
__device__ __forceinline__ float dw_sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }
// gate activations from one exp2 and one reciprocal each (v_exp_f32 / v_rcp_f32, ~1 ulp):
// sigmoid(x) = 1 / (1 + 2^(-x log2 e)), tanh(x) = 2 sigmoid(2x) - 1 (absolute error ~1e-7 near 0)
__device__ __forceinline__ float dw_sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
__device__ __forceinline__ float dw_tanh_fast(float x) {
  return 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -2.8853900817779268f)) - 1.0f;
}

// ---------------- noise-step embedding + diffusion projections of every layer ----------------
__global__ __launch_bounds__(512) void dw_embed_kernel(DWEmbedArgs a) {
  __shared__ float enc[128], h1[512], h2[512];
  const int r = blockIdx.x, tid = threadIdx.x;
  const float nl = a.noise_levels ? a.noise_levels[r] : (a.time_step_mode ? (float)r : a.table[r]);
  if (tid < 64) {                                   // diffwave.py:41-45
    const float v = nl * a.emb_vec[tid];
    enc[tid] = sinf(v);
    enc[tid + 64] = cosf(v);
  }
  __syncthreads();
  {
    float s = a.b1[tid];
    for (int k = 0; k < 128; ++k) s += a.w1[tid * 128 + k] * enc[k];
    h1[tid] = dw_silu(s);
  }
  __syncthreads();
  {
    float s = a.b2[tid];
    for (int k = 0; k < 512; ++k) s += a.w2[tid * 512 + k] * h1[k];
    h2[tid] = dw_silu(s);
  }
  __syncthreads();
  for (int o = tid; o < a.L * DW_C; o += 512) {    // diffusion_projection of every layer
    float s = a.pb[o];
    const float* w = a.pw + (size_t)o * 512;
    for (int k = 0; k < 512; ++k) s += w[k] * h2[k];
    a.out[(size_t)r * a.L * DW_C + o] = s;
  }
}

hipError_t launch_dw_embed(const DWEmbedArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(dw_embed_kernel, dim3(a.R), dim3(512), 0, s, a);
  return hipGetLastError();
}

// ---------------- SpectrogramUpsampler (ConvTranspose2d [3,32] stride [1,16] pad [1,8]) ----------------
// out(h, w) = bias + sum_{kh, kw} in(h + 1 - kh, (w + 8 - kw) / 16) k(kh, kw) over the kw with
// (w + 8 - kw) % 16 == 0, then leaky_relu(0.4)
__device__ __forceinline__ float dw_up_point(const float* in, int H, int Win, const float* k, float bias, int h, int w) {
  float s = bias;
  const int kw0 = (w + 8) & 15;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int hi = h + 1 - kh;
    if (hi < 0 || hi >= H) continue;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int kw = kw0 + 16 * m;
      const int wi = (w + 8 - kw) >> 4;
      if (wi < 0 || wi >= Win) continue;
      s += in[hi * Win + wi] * k[kh * 32 + kw];
    }
  }
  return s > 0.f ? s : s * 0.4f;
}

__global__ __launch_bounds__(256) void dw_upsample1_kernel(DWUpArgs a) {
  const int Wo = 16 * a.F;
  const int64_t total = (int64_t)a.B * a.H * Wo;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int w = (int)(i % Wo);
    const int64_t bh = i / Wo;
    const int h = (int)(bh % a.H), b = (int)(bh / a.H);
    a.mid[i] = dw_up_point(a.spec + (size_t)b * a.H * a.F, a.H, a.F, a.k1, a.b1[0], h, w);
  }
}

// second pass, written sample-major [B][N][Kp] in T (zero rows h >= H pad K to a multiple of 32):
// one thread per output sample n, all Kp values of it as 16-byte vectors; neighbouring lanes read
// the same or adjacent first-pass columns (coalesced)
template <typename T>
__global__ __launch_bounds__(256) void dw_upsample2_kernel(DWUpArgs a) {
  constexpr int VE = 16 / (int)sizeof(T);
  typedef T vec __attribute__((ext_vector_type(VE)));
  const int Wm = 16 * a.F, N = 256 * a.F;
  const int64_t total = (int64_t)a.B * N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int n = (int)(i % N), b = (int)(i / N);
    const float* mid = a.mid + (size_t)b * a.H * Wm;
    T* out = (T*)a.out + i * a.Kp;
    for (int h0 = 0; h0 < a.Kp; h0 += VE) {
      vec v;
#pragma unroll
      for (int j = 0; j < VE; ++j) {
        const int h = h0 + j;
        v[j] = from_f32<T>(h < a.H ? dw_up_point(mid, a.H, Wm, a.k2, a.b2[0], h, n) : 0.f);
      }
      *(vec*)(out + h0) = v;
    }
  }
}

hipError_t launch_dw_upsample(int dtype, const DWUpArgs& a, hipStream_t s) {
  if (a.Kp % 8) return hipErrorInvalidValue;
  const int64_t t1 = (int64_t)a.B * a.H * 16 * a.F, t2 = (int64_t)a.B * 256 * a.F;
  hipLaunchKernelGGL(dw_upsample1_kernel, dim3((unsigned)std::min<int64_t>((t1 + 255) / 256, 65535)), dim3(256), 0, s, a);
  const dim3 g2((unsigned)std::min<int64_t>((t2 + 255) / 256, 65535));
  if (dtype == DT_F32) hipLaunchKernelGGL(dw_upsample2_kernel<float>, g2, dim3(256), 0, s, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(dw_upsample2_kernel<bf16_t>, g2, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(dw_upsample2_kernel<f16_t>, g2, dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------- conditioner projections of all layers (step-invariant GEMM) ----------------
// cond[l][b][n][co] = sum_k Wc[l][co][k] spec[b][n][k] + bc[l][co]; block = 128 samples x 128 co.
// Block order: the L layer blocks of one sample tile are consecutive on one XCD (blocks i and i + 8
// share an XCD under round-robin dealing), so the tile's spectrogram rows (Kp up to 544 channels:
// 139 KB in 16 bits) come from HBM once and from that XCD's L2 for the other layers (tile-major
// over all layers at once re-read the whole 1.1 GB spectrogram per layer: 18 GB fetched, 17 ms)
template <typename T>
__global__ __launch_bounds__(256) void dw_cond_kernel(DWCondArgs a) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int tpc = (a.N + DW_MS - 1) / DW_MS, ntl = tpc * a.B;
  const int xcd = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int tile = xcd + 8 * (j / a.L), l = j - (j / a.L) * a.L;
  if (tile >= ntl) return;                          // block-uniform (padding of the last group of 8)
  const int b = tile / tpc, n0 = (tile - b * tpc) * DW_MS;
  const T* W = (const T*)a.w + (size_t)l * 128 * a.Kp;
  const T* S = (const T*)a.spec + (size_t)b * a.N * a.Kp;
  f32x4 acc[2][8];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
  const T* arow[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) arow[c] = W + (size_t)((wave * 2 + c) * 16 + (lane & 15)) * a.Kp + g * 8;
  const T* brow[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) brow[p] = S + (size_t)min(n0 + p * 16 + (lane & 15), a.N - 1) * a.Kp + g * 8;
  for (int k = 0; k < a.Kp; k += 32) {
    Frag<T> af[2], bf[8];
#pragma unroll
    for (int c = 0; c < 2; ++c) af[c] = load_frag<T>((const char*)(arow[c] + k));
#pragma unroll
    for (int p = 0; p < 8; ++p) bf[p] = load_frag<T>((const char*)(brow[p] + k));
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int p = 0; p < 8; ++p) mfma_frag(acc[c][p], af[c], bf[p]);
  }
  T* out = (T*)a.out;
  if constexpr (sizeof(T) == 2) {
    // the block's 128 x 128 tile goes through LDS so that HBM sees whole 256-byte rows (a contiguous
    // 32 KB run: out is [L][B][N][128]); 8-byte accumulator stores scatter 32-byte pieces
    constexpr int RS = 128 * 2 + 16;                 // padded row stride (bytes)
    __shared__ __attribute__((aligned(16))) char tl[DW_MS * RS];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int co = (wave * 2 + c) * 16 + 4 * g;
      float bias[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) bias[i] = a.bias[l * 128 + co + i];
#pragma unroll
      for (int p = 0; p < 8; ++p)
        store4<T>((T*)(tl + (p * 16 + (lane & 15)) * RS) + co, acc[c][p][0] + bias[0], acc[c][p][1] + bias[1],
                  acc[c][p][2] + bias[2], acc[c][p][3] + bias[3]);
    }
    __syncthreads();
    const int rows = min(DW_MS, a.N - n0);
    char* dst = (char*)(out + (((size_t)l * a.B + b) * a.N + n0) * 128);
#pragma unroll
    for (int k = 0; k < DW_MS * 16 / 256; ++k) {    // 16 x 16 B per row
      const int u = tid + k * 256, r = u >> 4, q = u & 15;
      if (r < rows) *(f32x4*)(dst + r * 256 + q * 16) = *(const f32x4*)(tl + r * RS + q * 16);
    }
  } else {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int co = (wave * 2 + c) * 16 + 4 * g;
      float bias[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) bias[i] = a.bias[l * 128 + co + i];
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        const int n = n0 + p * 16 + (lane & 15);
        if (n >= a.N) continue;
        store4<T>(out + (((size_t)l * a.B + b) * a.N + n) * 128 + co, acc[c][p][0] + bias[0], acc[c][p][1] + bias[1],
                  acc[c][p][2] + bias[2], acc[c][p][3] + bias[3]);
      }
    }
  }
}

hipError_t launch_dw_cond(int dtype, const DWCondArgs& a, hipStream_t s) {
  if (a.Kp % 32) return hipErrorInvalidValue;
  const int ntl = (a.N + DW_MS - 1) / DW_MS * a.B;
  const dim3 grid((unsigned)((ntl + 7) / 8 * 8 * a.L));
  if (dtype == DT_F32) hipLaunchKernelGGL(dw_cond_kernel<float>, grid, dim3(256), 0, s, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(dw_cond_kernel<bf16_t>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(dw_cond_kernel<f16_t>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------- input projection (diffwave.py:146-147) ----------------
template <typename T>
__global__ __launch_bounds__(256) void dw_input_kernel(DWInArgs a) {
  constexpr int VE = 16 / (int)sizeof(T);
  typedef T vec __attribute__((ext_vector_type(VE)));
  const int64_t total = a.total * (DW_C / VE);
  if (a.t_dev && blockIdx.x == 0 && threadIdx.x == 0) *a.t_dev -= 1;   // this step's t
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int q = (int)(i % (DW_C / VE));
    const float au = a.audio[i / (DW_C / VE)];
    vec v;
#pragma unroll
    for (int e = 0; e < VE; ++e) v[e] = from_f32<T>(fmaxf(a.w[q * VE + e] * au + a.b[q * VE + e], 0.f));
    *(vec*)((T*)a.x + i * VE) = v;
  }
}

hipError_t launch_dw_input(int dtype, const DWInArgs& a, hipStream_t s) {
  const dim3 grid((unsigned)std::min<int64_t>((a.total * 8 + 255) / 256, 8192));
  if (dtype == DT_F32) hipLaunchKernelGGL(dw_input_kernel<float>, grid, dim3(256), 0, s, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(dw_input_kernel<bf16_t>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(dw_input_kernel<f16_t>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------- fused residual layer ----------------
// PREW: the 16-bit weight fragments held in registers for the whole block (236 VGPRs: two blocks
// per CU); without, loaded per K step (three blocks per CU)
template <typename T, bool PREW>
__global__ __launch_bounds__(256, (PREW || sizeof(T) == 4) ? 2 : 3) void dw_layer_kernel(DWLayerArgs a) {
  constexpr int ES = (int)sizeof(T), VE = 16 / ES;
  constexpr int UPS = DW_C / VE;                  // 16-byte units (planes) per sample and tap
  constexpr int PB = 64 / UPS;                    // samples per 64-unit staging group
  constexpr int PLANE = DW_MS * 16;               // bytes per plane (2 KB, = 0 mod 256)
  constexpr int MAXU = 12;
  typedef T vec4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* yin = smem;                               // [3 taps][UPS][128 samples][16 B]
  char* zl = smem;                                // [UPS][128 samples][16 B], aliases yin after GEMM 1
  constexpr int XS = DW_C * ES + 16;              // residual row stride (16-byte aligned, staggers banks)
  char* xl = smem + 3 * UPS * PLANE;              // [128 samples][XS]: raw x of the tile (residual)

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int N = a.N, d = a.dil;
  const int cg = wave * 16 + 4 * g;               // gate row base; filter rows cg + 64
  // both GEMMs' weight fragments and biases are issued first (16-bit weights: 14 fragments x 4
  // VGPRs; fp32 fragments are twice that, so the fp32 path loads them per K step)
  const T* w1 = (const T*)a.w1;
  const T* w2 = (const T*)a.w2;
  constexpr bool PRE = sizeof(T) == 2 && PREW;
  auto w1frag = [&](int s, int c) {
    return load_frag<T>((const char*)(w1 + (size_t)(c * 64 + wave * 16 + (lane & 15)) * 192 + s * 32 + g * 8));
  };
  auto w2frag = [&](int s) { return load_frag<T>((const char*)(w2 + (size_t)(wave * 16 + (lane & 15)) * DW_C + s * 32 + g * 8)); };
  Frag<T> aw1[PRE ? 6 : 1][2], aw2[PRE ? 2 : 1];
  if constexpr (PRE) {
#pragma unroll
    for (int s = 0; s < 6; ++s)
#pragma unroll
      for (int c = 0; c < 2; ++c) aw1[s][c] = w1frag(s, c);
#pragma unroll
    for (int s = 0; s < 2; ++s) aw2[s] = w2frag(s);
  }
  float bg[4], bfl[4], br[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { bg[i] = a.b1[cg + i]; bfl[i] = a.b1[cg + 64 + i]; br[i] = a.b2[cg + i]; }
  const int t_now = a.t_dev ? *a.t_dev : 0;
  {
  // plain order: round-robin dealing spreads a clip's neighbouring tiles over the XCDs (measured
  // faster than the XCD-contiguous order of the conv kernels: 216.6 vs 228.6 us per layer)
  const int b = blockIdx.y, n0 = blockIdx.x * DW_MS;
  const T* xin = (const T*)a.x_in + (size_t)b * N * DW_C;
  const float* ds = a.ds + ((size_t)(a.ds_per_b ? b : t_now) * a.L + a.layer) * DW_C;
  // the diffusion projection of this thread's staging channels first (needed first: the loads
  // issued after it stay in flight while the staging waits for it); the channel unit q of a
  // staging unit depends on tid only (u = u0 + tid + 256 k with u0 a multiple of 256)
  const int qs = (tid & 63) / PB;
  float dsv[VE];
#pragma unroll
  for (int e = 0; e < VE; ++e) dsv[e] = ds[qs * VE + e];
  // then every other load that does not depend on the staged image, so a tile waits on memory
  // once: the conditioner rows of this lane's gate / filter channels (used after GEMM 1) and the
  // residual x of its output channels (used in the epilogue); clamped, unconditional
  vec4 cnd[2][8];
  {
    const T* cb = (const T*)a.cond + (size_t)a.layer * a.B * N * 128;   // layer-major: one stream per layer
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int n = min(n0 + p * 16 + (lane & 15), N - 1);
      const T* cp = cb + ((size_t)b * N + n) * 128;
      cnd[0][p] = *(const vec4*)(cp + cg);
      cnd[1][p] = *(const vec4*)(cp + cg + 64);
    }
  }
  // ---- 1. y = x + diffusion projection -> LDS ----
  // dilation <= 64: one window of rows n0 - d .. n0 + 127 + d (the three taps overlap; each x row
  // is read and transformed once), planes padded to 256 B; larger dilations: three disjoint tap
  // images of 128 rows
  const bool win = d <= 64;
  const int ROWS = win ? (DW_MS + 2 * d + PB - 1) / PB * PB : DW_MS, TAPS = win ? 1 : 3;   // whole staging groups
  const int PL = win ? (ROWS * 16 + 255) / 256 * 256 : PLANE;
  const int NUr = TAPS * ROWS * UPS;             // 16-bit: <= MAXU * 256 (checked by the launcher)
  auto stage_pass = [&](int u0) {
    f32x4 reg[MAXU];
    int dst[MAXU], qv[MAXU], xr[MAXU];
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = min(u0 + tid + k * 256, NUr - 1);
      const int tap = u / (ROWS * UPS), r = u - tap * (ROWS * UPS);
      const int grp = r >> 6, j = r & 63, q = j / PB, s = grp * PB + (j % PB);
      const int n = win ? n0 - d + s : n0 + s + (tap - 1) * d;
      const bool ok = n >= 0 && n < N && u0 + tid + k * 256 < NUr;
      reg[k] = *(const f32x4*)(xin + (size_t)min(max(n, 0), N - 1) * DW_C + q * VE);
      dst[k] = (u0 + tid + k * 256 < NUr) ? ((tap * UPS + q) * PL + s * 16) : -1;
      qv[k] = ok ? 1 : 0;
      // the centre rows n0 .. n0+127 also go to the residual image, raw
      const int c = n - n0;
      xr[k] = (u0 + tid + k * 256 < NUr && (win || tap == 1) && c >= 0 && c < DW_MS) ? c * XS + q * 16 : -1;
    }
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      typedef T vec __attribute__((ext_vector_type(VE)));
      if (xr[k] >= 0) *(f32x4*)(xl + xr[k]) = reg[k];
      vec v = __builtin_bit_cast(vec, reg[k]);
#pragma unroll
      for (int e = 0; e < VE; ++e) v[e] = from_f32<T>(qv[k] ? to_f32<T>(v[e]) + dsv[e] : 0.f);
      if (dst[k] >= 0) *(f32x4*)(yin + dst[k]) = __builtin_bit_cast(f32x4, v);
    }
  };
  if constexpr (ES == 2) stage_pass(0);            // straight-line: the loads above stay in flight
  else
    for (int u0 = 0; u0 < NUr; u0 += MAXU * 256) stage_pass(u0);
  lds_sync();                                      // (the conditioner / residual loads stay in flight)
  // ---- 2. dilated conv GEMM: rows {16w.., 64+16w..} x 128 samples, K = 192 ----
  f32x4 acc[2][8];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int tap = s >> 1, half = s & 1;
    Frag<T> af[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) af[c] = PRE ? aw1[PRE ? s : 0][c] : w1frag(s, c);
    const char* pb = yin + ((win ? 0 : tap * UPS) + (half * 32 + g * 8) / VE) * PL +
                     ((win ? tap * d : 0) + (lane & 15)) * 16;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const Frag<T> bf = load_planes<T>(pb + p * 256, PL);
#pragma unroll
      for (int c = 0; c < 2; ++c) mfma_frag(acc[c][p], af[c], bf);
    }
  }
  // ---- gated activation z = sigmoid(gate) * tanh(filter) -> LDS (plane-major, over yin) ----
  lds_sync();                                      // every wave is done reading yin
  {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      float z[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float gate = acc[0][p][i] + bg[i] + to_f32<T>(cnd[0][p][i]);
        const float filt = acc[1][p][i] + bfl[i] + to_f32<T>(cnd[1][p][i]);
        z[i] = dw_sigmoid_fast(gate) * dw_tanh_fast(filt);
      }
      char* zp = zl + (cg / VE) * PLANE + (p * 16 + (lane & 15)) * 16 + (cg % VE) * ES;
      store4<T>((T*)zp, z[0], z[1], z[2], z[3]);
      const int n = n0 + p * 16 + (lane & 15);      // z of every layer, for the deferred skip GEMM
      if (n0 + DW_MS <= N || n < N) store4<T>((T*)a.z + (((size_t)a.layer * a.B + b) * N + n) * DW_C + cg, z[0], z[1], z[2], z[3]);
    }
  }
  lds_sync();                                      // (the z stores stay in flight)
  // ---- 3. output_residual GEMM: rows 16w.., K = 64 (output_projection is deferred: dw_skip_kernel) ----
#pragma unroll
  for (int p = 0; p < 8; ++p) acc[0][p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const Frag<T> af = PRE ? aw2[PRE ? s : 0] : w2frag(s);
    const char* pb = zl + ((s * 32 + g * 8) / VE) * PLANE + (lane & 15) * 16;
#pragma unroll
    for (int p = 0; p < 8; ++p) mfma_frag(acc[0][p], af, load_planes<T>(pb + p * 256, PLANE));
  }
  // ---- epilogue: x_out = (x + residual) / sqrt(2) ----
  {
    // (x + residual) / sqrt(2) (diffwave.py:108): the fp32 path divides like the reference; the
    // 16-bit paths multiply by the reciprocal (<= 1 ulp of fp32 before the storage rounding)
    const float r2 = 1.41421353816986083984375f;   // (float)sqrt(2.0)
    const float ir2 = 0.707106769084930419921875f;  // (float)(1 / sqrt(2.0))
    auto scale = [&](float v) { return sizeof(T) == 4 ? v / r2 : v * ir2; };
    T* xo = (T*)a.x_out + (size_t)b * N * DW_C;
    const bool full = n0 + DW_MS <= N;              // block-uniform: no per-row checks
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int n = n0 + p * 16 + (lane & 15);
      if (!full && n >= N) continue;
      const vec4 xv = *(const vec4*)(xl + (p * 16 + (lane & 15)) * XS + cg * ES);
      store4<T>(xo + (size_t)n * DW_C + cg, scale(to_f32<T>(xv[0]) + (acc[0][p][0] + br[0])),
                scale(to_f32<T>(xv[1]) + (acc[0][p][1] + br[1])), scale(to_f32<T>(xv[2]) + (acc[0][p][2] + br[2])),
                scale(to_f32<T>(xv[3]) + (acc[0][p][3] + br[3])));
    }
  }
  }
}

// ---------------- GEMM-group tile body shared by the ping-pong and dilation-chain layers ----------------
template <typename T> using dw_v4 = T __attribute__((ext_vector_type(4)));

// conditioner rows (gate cg.., filter cg+64..) of FPW 16-sample fragments from p0 of tile (b, n0)
template <typename T, int FPW>
__device__ __forceinline__ void dw_cond_rows(const DWLayerArgs& a, int b, int n0, int p0, int cg, int lane,
                                             dw_v4<T> (&cnd)[2][FPW]) {
  const int N = a.N;
  const T* cb = (const T*)a.cond + (size_t)a.layer * a.B * N * 128;   // layer-major: one stream per layer
#pragma unroll
  for (int p = 0; p < FPW; ++p) {
    const int n = min(n0 + (p0 + p) * 16 + (lane & 15), N - 1);
    const T* cp = cb + ((size_t)b * N + n) * 128;
    cnd[0][p] = *(const dw_v4<T>*)(cp + cg);
    cnd[1][p] = *(const dw_v4<T>*)(cp + cg + 64);
  }
}

// part 1: dilated-conv GEMM over the three tap images tb[t] (plane stride PL), gate, z -> LDS zl and
// to the layer's z rows (deferred skip GEMM)
template <typename T, int FPW>
__device__ __forceinline__ void dw_tile_gate(const DWLayerArgs& a, const char* const (&tb)[3], int PL, char* zl, int b,
                                             int n0, int p0, int cg, int lane, const Frag<T> (&aw1)[6][2],
                                             const float (&bg)[4], const float (&bfl)[4],
                                             const dw_v4<T> (&cnd)[2][FPW]) {
  constexpr int VE = 8, ES = 2, PLANE = DW_MS * 16;
  const int N = a.N, g = lane >> 4;
  f32x4 acc[2][FPW];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int p = 0; p < FPW; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const int tap = s >> 1, half = s & 1;
    const char* pb = tb[tap] + ((half * 32 + g * 8) / VE) * PL + (lane & 15) * 16;
#pragma unroll
    for (int p = 0; p < FPW; ++p) {
      const Frag<T> bf = load_planes<T>(pb + (p0 + p) * 256, PL);
#pragma unroll
      for (int c = 0; c < 2; ++c) mfma_frag(acc[c][p], aw1[s][c], bf);
    }
  }
  const bool full = n0 + DW_MS <= N;
#pragma unroll
  for (int p = 0; p < FPW; ++p) {
    float z[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float gate = acc[0][p][i] + bg[i] + to_f32<T>(cnd[0][p][i]);
      const float filt = acc[1][p][i] + bfl[i] + to_f32<T>(cnd[1][p][i]);
      z[i] = dw_sigmoid_fast(gate) * dw_tanh_fast(filt);
    }
    store4<T>((T*)(zl + (cg / VE) * PLANE + ((p0 + p) * 16 + (lane & 15)) * 16 + (cg % VE) * ES), z[0], z[1], z[2], z[3]);
    const int n = n0 + (p0 + p) * 16 + (lane & 15);
    if (full || n < N) store4<T>((T*)a.z + (((size_t)a.layer * a.B + b) * N + n) * DW_C + cg, z[0], z[1], z[2], z[3]);
  }
}

// part 2: output_residual GEMM from zl, epilogue (x + residual) / sqrt(2) with the raw rows xl
template <typename T, int FPW>
__device__ __forceinline__ void dw_tile_out(const DWLayerArgs& a, const char* zl, const char* xl, int b, int n0, int p0,
                                            int cg, int lane, const Frag<T> (&aw2)[2], const float (&br)[4]) {
  constexpr int VE = 8, ES = 2, PLANE = DW_MS * 16, XS = DW_C * ES + 16;
  const int N = a.N, g = lane >> 4;
  const float ir2 = 0.707106769084930419921875f;   // (float)(1 / sqrt(2.0)), as dw_layer_kernel's 16-bit path
  f32x4 acc[FPW];
#pragma unroll
  for (int p = 0; p < FPW; ++p) acc[p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const char* pb = zl + ((s * 32 + g * 8) / VE) * PLANE + (lane & 15) * 16;
#pragma unroll
    for (int p = 0; p < FPW; ++p) mfma_frag(acc[p], aw2[s], load_planes<T>(pb + (p0 + p) * 256, PLANE));
  }
  const bool full = n0 + DW_MS <= N;
  T* xo = (T*)a.x_out + (size_t)b * N * DW_C;
#pragma unroll
  for (int p = 0; p < FPW; ++p) {
    const int n = n0 + (p0 + p) * 16 + (lane & 15);
    if (!full && n >= N) continue;
    const dw_v4<T> xv = *(const dw_v4<T>*)(xl + ((p0 + p) * 16 + (lane & 15)) * XS + cg * ES);
    store4<T>(xo + (size_t)n * DW_C + cg, (to_f32<T>(xv[0]) + (acc[p][0] + br[0])) * ir2,
              (to_f32<T>(xv[1]) + (acc[p][1] + br[1])) * ir2, (to_f32<T>(xv[2]) + (acc[p][2] + br[2])) * ir2,
              (to_f32<T>(xv[3]) + (acc[p][3] + br[3])) * ir2);
  }
}

// the GEMM group's registers: both GEMMs' weight fragments and biases of channel quarter wq
template <typename T>
__device__ __forceinline__ void dw_gemm_regs(const DWLayerArgs& a, int wq, int lane, Frag<T> (&aw1)[6][2],
                                             Frag<T> (&aw2)[2], float (&bg)[4], float (&bfl)[4], float (&br)[4]) {
  const int g = lane >> 4, cg = wq * 16 + 4 * g;
  const T* w1 = (const T*)a.w1;
  const T* w2 = (const T*)a.w2;
#pragma unroll
  for (int s = 0; s < 6; ++s)
#pragma unroll
    for (int c = 0; c < 2; ++c)
      aw1[s][c] = load_frag<T>((const char*)(w1 + (size_t)(c * 64 + wq * 16 + (lane & 15)) * 192 + s * 32 + g * 8));
#pragma unroll
  for (int s = 0; s < 2; ++s) aw2[s] = load_frag<T>((const char*)(w2 + (size_t)(wq * 16 + (lane & 15)) * DW_C + s * 32 + g * 8));
#pragma unroll
  for (int i = 0; i < 4; ++i) { bg[i] = a.b1[cg + i]; bfl[i] = a.b1[cg + 64 + i]; br[i] = a.b2[cg + i]; }
}

// ---------------- ping-pong residual layer (16-bit) ----------------
// The same layer as dw_layer_kernel, with the staging and the GEMMs of a CU split between two wave
// groups that work on different tiles: a persistent block of 8 waves walks a strided list of
// 128-sample tiles; waves 4-7 (staging group) load tile k+1 -- y = x + diffusion projection over the
// dilated window, the raw residual rows -- into one of two LDS slots while waves 0-3 (GEMM group) run
// tile k's dilated-conv GEMM, gated activation, output_residual GEMM and epilogue from the other.
// Two workgroup barriers per tile: the GEMM group's z hand-off (z goes to its own LDS buffer) and
// the slot swap.  The staging group's global loads are in flight during the GEMM group's MFMAs, so
// a CU waits on memory only when a tile's loads outlast its GEMMs.
constexpr int DW_PP_Y = 3 * 8 * DW_MS * 16;                  // yin: 3 taps x 8 planes x 128 samples (16-bit)
constexpr int DW_PP_SLOT = DW_PP_Y + DW_MS * (DW_C * 2 + 16);  // + raw residual rows
constexpr int DW_PP_LDS = 2 * DW_PP_SLOT + 8 * DW_MS * 16;     // two slots + z [8 planes][128][16 B]

template <typename T, int GW>
__global__ __launch_bounds__(64 * (GW + 4), 1) void dw_layer_pp_kernel(DWLayerArgs a) {
  static_assert(sizeof(T) == 2 && (GW == 4 || GW == 8), "16-bit, 4 or 8 GEMM waves");
  constexpr int FPW = 8 * 4 / GW;                  // 16-sample fragments per GEMM wave
  constexpr int ES = 2, VE = 8, UPS = 8, PB = 8;  // 16-byte units per sample; samples per 64-unit group
  constexpr int PLANE = DW_MS * 16, XS = DW_C * ES + 16, MAXU = 12;
  typedef T vec4 __attribute__((ext_vector_type(4)));
  typedef T vec __attribute__((ext_vector_type(VE)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* zl = smem + 2 * DW_PP_SLOT;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int N = a.N, d = a.dil, G = gridDim.x;
  const int tpc = (N + DW_MS - 1) / DW_MS, ntiles = tpc * a.B;
  const int t_now = a.t_dev ? *a.t_dev : 0;
  const bool win = d <= 64;
  const int ROWS = win ? (DW_MS + 2 * d + PB - 1) / PB * PB : DW_MS, TAPS = win ? 1 : 3;
  const int PL = win ? (ROWS * 16 + 255) / 256 * 256 : PLANE;
  const int NUr = TAPS * ROWS * UPS;               // <= MAXU * 256 (checked by the launcher)
  int tile = blockIdx.x;

  if (wave >= GW) {
    // ---------------- staging group ----------------
    const int st = tid - 64 * GW;                      // 0 .. 255
    const int qs = (st & 63) / PB;                 // channel unit of every unit this thread stages
    f32x4 reg[MAXU];
    float dsv[VE];
    auto issue = [&](int tl) {                     // global loads of tile tl into registers
      const int b = tl / tpc, n0 = (tl - b * tpc) * DW_MS;
      const T* xin = (const T*)a.x_in + (size_t)b * N * DW_C;
      const float* ds = a.ds + ((size_t)(a.ds_per_b ? b : t_now) * a.L + a.layer) * DW_C;
#pragma unroll
      for (int e = 0; e < VE; ++e) dsv[e] = ds[qs * VE + e];
#pragma unroll
      for (int k = 0; k < MAXU; ++k) {
        const int u = min(st + k * 256, NUr - 1);
        const int tap = u / (ROWS * UPS), r = u - tap * (ROWS * UPS);
        const int grp = r >> 6, j = r & 63, q = j / PB, s = grp * PB + (j % PB);
        const int n = win ? n0 - d + s : n0 + s + (tap - 1) * d;
        reg[k] = *(const f32x4*)(xin + (size_t)min(max(n, 0), N - 1) * DW_C + q * VE);
      }
    };
    auto land = [&](int tl, char* slot) {          // transform + LDS stores (same unit map as issue)
      const int b = tl / tpc, n0 = (tl - b * tpc) * DW_MS;
      (void)b;
      char* yin = slot;
      char* xl = slot + DW_PP_Y;
#pragma unroll
      for (int k = 0; k < MAXU; ++k) {
        const int u = st + k * 256;
        if (u < NUr) {
          const int tap = u / (ROWS * UPS), r = u - tap * (ROWS * UPS);
          const int grp = r >> 6, j = r & 63, q = j / PB, s = grp * PB + (j % PB);
          const int n = win ? n0 - d + s : n0 + s + (tap - 1) * d;
          const bool ok = n >= 0 && n < N;
          const int c = n - n0;                    // the centre rows also go to the residual image, raw
          if ((win || tap == 1) && c >= 0 && c < DW_MS) *(f32x4*)(xl + c * XS + q * 16) = reg[k];
          vec v = __builtin_bit_cast(vec, reg[k]);
#pragma unroll
          for (int e = 0; e < VE; ++e) v[e] = from_f32<T>(ok ? to_f32<T>(v[e]) + dsv[e] : 0.f);
          *(f32x4*)(yin + (tap * UPS + q) * PL + s * 16) = __builtin_bit_cast(f32x4, v);
        }
      }
    };
    // (a second register set, issuing tile k+2 while tile k+1 lands, measured no faster: 193.4 vs
    // 190.5 us per layer at config #3)
    if (tile < ntiles) { issue(tile); land(tile, smem); }
    lds_sync();
    for (int k = 0; tile < ntiles; ++k, tile += G) {
      const int next = tile + G;
      if (next < ntiles) issue(next);
      lds_sync();                                  // (the GEMM group's z hand-off; the loads stay in flight)
      if (next < ntiles) land(next, smem + ((k + 1) & 1) * DW_PP_SLOT);
      lds_sync();                                  // slot swap
    }
    return;
  }

  // ---------------- GEMM group: wave = channel quarter wq x sample part (FPW fragments from p0) ----------------
  const int wq = wave & 3, p0 = (wave >> 2) * FPW;
  const int cg = wq * 16 + 4 * g;                // gate rows cg..cg+3; filter rows cg + 64
  Frag<T> aw1[6][2], aw2[2];
  float bg[4], bfl[4], br[4];
  dw_gemm_regs<T>(a, wq, lane, aw1, aw2, bg, bfl, br);
  // conditioner rows of this wave's channels: loaded one tile ahead (issued after the gate of the
  // previous tile, so they are in flight during its output_residual GEMM, epilogue and barriers)
  dw_v4<T> cnd[2][FPW];
  if (tile < ntiles) dw_cond_rows<T, FPW>(a, tile / tpc, (tile % tpc) * DW_MS, p0, cg, lane, cnd);
  lds_sync();                                      // tile 0 staged
  for (int k = 0; tile < ntiles; ++k, tile += G) {
    const int b = tile / tpc, n0 = (tile - b * tpc) * DW_MS;
    const char* yin = smem + (k & 1) * DW_PP_SLOT;
    const char* tb[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) tb[t] = yin + (win ? t * d * 16 : t * UPS * PL);
    dw_tile_gate<T, FPW>(a, tb, PL, zl, b, n0, p0, cg, lane, aw1, bg, bfl, cnd);
    if (tile + G < ntiles) dw_cond_rows<T, FPW>(a, (tile + G) / tpc, ((tile + G) % tpc) * DW_MS, p0, cg, lane, cnd);
    lds_sync();                                    // z hand-off (the z stores and next conditioner loads stay in flight)
    dw_tile_out<T, FPW>(a, zl, yin + DW_PP_Y, b, n0, p0, cg, lane, aw2, br);
    lds_sync();                                    // slot swap
  }
}

// ---------------- dilation-chain residual layer (16-bit, dilation a multiple of 128) ----------------
// For d >= 128 the three taps of a 128-sample tile are three disjoint 128-row images, so a tile of
// the ping-pong kernel stages three images.  Here a block walks a dilation chain -- tiles n0, n0 + d,
// n0 + 2d, ... of one clip, whose taps are images n0 - d, n0, n0 + d -- in segments of DW_CH_SEG
// tiles and keeps the images in a ring of four LDS slots: after a segment's first tile every tile
// stages ONE new image (its successor's +d tap), the GEMM group reads the other three.  An image
// slot also holds the raw rows (the residual, when the image is a tile's centre).  Same wave groups,
// barriers and GEMM-group body as the ping-pong kernel.  A segment's first tile waits for its three
// images (no overlap), so segments are long: d >= 128 layers 213 -> 199 / 190 / 185 us at 8 / 16 /
// 32 tiles per segment (config #3; the d <= 64 ping-pong layers: 182-189 us).
constexpr int DW_CH_IMG = 8 * DW_MS * 16;                      // y image: 8 planes x 128 rows x 16 B
constexpr int DW_CH_SLOT = DW_CH_IMG + DW_MS * (DW_C * 2 + 16);  // + raw rows
constexpr int DW_CH_LDS = 4 * DW_CH_SLOT + 8 * DW_MS * 16;      // ring of four + z

template <typename T, int DW_CH_SEG>                           // tiles per chain segment
__global__ __launch_bounds__(512, 1) void dw_layer_chain_kernel(DWLayerArgs a) {
  static_assert(sizeof(T) == 2, "16-bit only");
  constexpr int VE = 8, PB = 8, PLANE = DW_MS * 16, XS = DW_C * 2 + 16, FPW = 8;
  typedef T vec __attribute__((ext_vector_type(VE)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* zl = smem + 4 * DW_CH_SLOT;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int N = a.N, d = a.dil, G = gridDim.x;
  const int tpc = (N + DW_MS - 1) / DW_MS, R = d / DW_MS;          // chains per clip
  const int t_now = a.t_dev ? *a.t_dev : 0;
  // segments per clip: chain rho has ceil((tpc - rho) / R) tiles
  int spc = 0;
  for (int rho = 0; rho < R && rho < tpc; ++rho) spc += ((tpc - rho + R - 1) / R + DW_CH_SEG - 1) / DW_CH_SEG;
  const int nseg = spc * a.B;
  // segment id -> clip b, chain rho, first chain index j0, tile count len
  auto segment = [&](int sid, int& b, int& rho, int& j0, int& len) {
    b = sid / spc;
    int r = sid - b * spc;
    rho = 0;
    for (;; ++rho) {
      const int nj = (tpc - rho + R - 1) / R, ns = (nj + DW_CH_SEG - 1) / DW_CH_SEG;
      if (r < ns) { j0 = r * DW_CH_SEG; len = min(DW_CH_SEG, nj - j0); return; }
      r -= ns;
    }
  };
  // image m of a segment (m = -1 .. len): rows nb + m d with nb = the first tile's n0; ring slot (m + 1) & 3
  auto slot = [&](int m) { return smem + ((m + 1) & 3) * DW_CH_SLOT; };

  if (wave >= 4) {
    // ---------------- staging group: one 1024-unit image = 4 units per thread ----------------
    const int st = tid - 256;
    const int qs = (st & 63) / PB;
    f32x4 reg[12];
    float dsv[VE];
    // loads of images m0 .. m0 + cnt - 1 (cnt <= 3) into reg[4 i ..]
    auto issue = [&](const T* xin, int nb, int m0, int cnt) {
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        if (k / 4 < cnt) {
          const int u = st + (k & 3) * 256, grp = u >> 6, j = u & 63, q = j / PB, s = grp * PB + (j % PB);
          const int n = nb + (m0 + k / 4) * d + s;
          reg[k] = *(const f32x4*)(xin + (size_t)min(max(n, 0), N - 1) * DW_C + q * VE);
        }
      }
    };
    auto land = [&](int nb, int m0, int cnt) {
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        if (k / 4 < cnt) {
          const int u = st + (k & 3) * 256, grp = u >> 6, j = u & 63, q = j / PB, s = grp * PB + (j % PB);
          const int m = m0 + k / 4, n = nb + m * d + s;
          const bool ok = n >= 0 && n < N;
          char* sl = slot(m);
          *(f32x4*)(sl + DW_CH_IMG + s * XS + q * 16) = reg[k];
          vec v = __builtin_bit_cast(vec, reg[k]);
#pragma unroll
          for (int e = 0; e < VE; ++e) v[e] = from_f32<T>(ok ? to_f32<T>(v[e]) + dsv[e] : 0.f);
          *(f32x4*)(sl + q * PLANE + s * 16) = __builtin_bit_cast(f32x4, v);
        }
      }
    };
    for (int sid = blockIdx.x; sid < nseg; sid += G) {
      int b, rho, j0, len;
      segment(sid, b, rho, j0, len);
      const int nb = (rho + j0 * R) * DW_MS;
      const T* xin = (const T*)a.x_in + (size_t)b * N * DW_C;
      const float* ds = a.ds + ((size_t)(a.ds_per_b ? b : t_now) * a.L + a.layer) * DW_C;
#pragma unroll
      for (int e = 0; e < VE; ++e) dsv[e] = ds[qs * VE + e];
      issue(xin, nb, -1, 3);                       // images -1, 0, 1: the first tile's taps
      land(nb, -1, 3);
      lds_sync();                                  // segment start
      for (int i = 0; i < len; ++i) {
        if (i + 1 < len) issue(xin, nb, i + 2, 1);
        lds_sync();                                // (the GEMM group's z hand-off; the loads stay in flight)
        if (i + 1 < len) land(nb, i + 2, 1);
        lds_sync();                                // tile done
      }
    }
    return;
  }

  // ---------------- GEMM group ----------------
  const int wq = wave & 3, p0 = 0;
  const int cg = wq * 16 + 4 * g;
  Frag<T> aw1[6][2], aw2[2];
  float bg[4], bfl[4], br[4];
  dw_gemm_regs<T>(a, wq, lane, aw1, aw2, bg, bfl, br);
  dw_v4<T> cnd[2][FPW];
  for (int sid = blockIdx.x; sid < nseg; sid += G) {
    int b, rho, j0, len;
    segment(sid, b, rho, j0, len);
    const int nb = (rho + j0 * R) * DW_MS;
    dw_cond_rows<T, FPW>(a, b, nb, p0, cg, lane, cnd);
    lds_sync();                                    // segment start: the first tile's images staged
    for (int i = 0; i < len; ++i) {
      const int n0 = nb + i * d;
      const char* tb[3] = {slot(i - 1), slot(i), slot(i + 1)};
      dw_tile_gate<T, FPW>(a, tb, PLANE, zl, b, n0, p0, cg, lane, aw1, bg, bfl, cnd);
      if (i + 1 < len) dw_cond_rows<T, FPW>(a, b, n0 + d, p0, cg, lane, cnd);
      lds_sync();                                  // z hand-off
      dw_tile_out<T, FPW>(a, zl, slot(i) + DW_CH_IMG, b, n0, p0, cg, lane, aw2, br);
      lds_sync();                                  // tile done
    }
  }
}

size_t dw_layer_lds_bytes(int dtype) {
  const int es = dtype == DT_F32 ? 4 : 2, ups = DW_C * es / 16;
  return (size_t)3 * ups * DW_MS * 16 + (size_t)DW_MS * (DW_C * es + 16);   // staging + residual rows
}

hipError_t launch_dw_layer(int dtype, const DWLayerArgs& a, hipStream_t s) {
  const dim3 grid((a.N + DW_MS - 1) / DW_MS, a.B);
  {  // the staging of one block fits a single pass of 12 units per thread
    const int ups = DW_C * (dtype == DT_F32 ? 4 : 2) / 16, pb = 64 / ups;
    const bool win = a.dil <= 64;
    const int rows = win ? (DW_MS + 2 * a.dil + pb - 1) / pb * pb : DW_MS;
    if (dtype != DT_F32 && (win ? 1 : 3) * rows * ups > 12 * 256) return hipErrorInvalidValue;
  }
  // 16-bit: the ping-pong kernel (config #3: 215.5 -> 190.5 us per layer); SDDM_DW_NOPP=1 runs the
  // one-phase kernel (A/B knob)
  static const bool nopp = std::getenv("SDDM_DW_NOPP") != nullptr;
  if (!nopp && dtype != DT_F32) {
    static int ncu = 0;
    if (!ncu) {
      int dev = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
        return hipErrorInvalidValue;
    }
    const int ntiles = (int)grid.x * (int)grid.y;
    const dim3 pgrid(ntiles < ncu ? ntiles : ncu);
    static const bool nochain = std::getenv("SDDM_DW_NOCHAIN") != nullptr;   // A/B knob
    if (!nochain && a.dil % DW_MS == 0) {          // dilation chains (d >= 128)
      static const int seg = std::getenv("SDDM_DW_CHSEG") ? std::atoi(std::getenv("SDDM_DW_CHSEG")) : 32;   // A/B knob (8 / 16 / 32)
      const int tpc = (a.N + DW_MS - 1) / DW_MS, R = a.dil / DW_MS;
      int spc = 0;
      for (int rho = 0; rho < R && rho < tpc; ++rho) spc += ((tpc - rho + R - 1) / R + seg - 1) / seg;
      const int nseg = spc * a.B;
      const dim3 cgrid(nseg < ncu ? nseg : ncu);
#define SDDM_DW_CHAIN(S)                                                                                          \
  if (dtype == DT_BF16) hipLaunchKernelGGL((dw_layer_chain_kernel<bf16_t, S>), cgrid, dim3(512), DW_CH_LDS, s, a); \
  else hipLaunchKernelGGL((dw_layer_chain_kernel<f16_t, S>), cgrid, dim3(512), DW_CH_LDS, s, a);
      if (seg == 32) { SDDM_DW_CHAIN(32) }
      else if (seg == 16) { SDDM_DW_CHAIN(16) }
      else { SDDM_DW_CHAIN(8) }
#undef SDDM_DW_CHAIN
      return hipGetLastError();
    }
    if (dtype == DT_BF16) hipLaunchKernelGGL((dw_layer_pp_kernel<bf16_t, 4>), pgrid, dim3(512), DW_PP_LDS, s, a);
    else hipLaunchKernelGGL((dw_layer_pp_kernel<f16_t, 4>), pgrid, dim3(512), DW_PP_LDS, s, a);
    return hipGetLastError();
  }
  const size_t lds = dw_layer_lds_bytes(dtype);
  static const bool nopre = std::getenv("SDDM_DW_NOPRE") != nullptr;   // experiment knob
  if (dtype == DT_F32) hipLaunchKernelGGL((dw_layer_kernel<float, false>), grid, dim3(256), lds, s, a);
  else if (dtype == DT_BF16) {
    if (nopre) hipLaunchKernelGGL((dw_layer_kernel<bf16_t, false>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((dw_layer_kernel<bf16_t, true>), grid, dim3(256), lds, s, a);
  } else {
    if (nopre) hipLaunchKernelGGL((dw_layer_kernel<f16_t, false>), grid, dim3(256), lds, s, a);
    else hipLaunchKernelGGL((dw_layer_kernel<f16_t, true>), grid, dim3(256), lds, s, a);
  }
  return hipGetLastError();
}

// ---------------- deferred skip sum: skip[b][n][co] = sum_l Wo_l z_l + sum_l bo_l (K = L x 64) ----------------
// diffwave.py:104-106, 150-152: every layer's output_projection applied to its stored gated
// activation z_l (layer-major [L][B][N][64]) in one GEMM instead of a per-layer fp32 read-modify-write.
template <typename T>
__global__ __launch_bounds__(256) void dw_skip_kernel(DWSkipArgs a) {
  // block = 256 samples; wave w owns samples [64 w, +64) x all 64 channels (4 x 4 MFMA tiles), so
  // every z fragment is read from HBM exactly once and the weight fragments come from L2
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int n0 = blockIdx.x * 256 + wave * 64, b = blockIdx.y, K = a.L * DW_C;
  const size_t LS = (size_t)a.B * a.N * DW_C;        // z is layer-major: [L][B][N][64]
  const T* Z = (const T*)a.z + (size_t)b * a.N * DW_C;
  const T* arow[4];
  const T* brow[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) arow[c] = (const T*)a.w + (size_t)(c * 16 + (lane & 15)) * K + g * 8;
#pragma unroll
  for (int p = 0; p < 4; ++p) brow[p] = Z + (size_t)min(n0 + p * 16 + (lane & 15), a.N - 1) * DW_C + g * 8;
  f32x4 acc[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
  Frag<T> af[4], bf[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) af[c] = load_frag<T>((const char*)arow[c]);
#pragma unroll
  for (int p = 0; p < 4; ++p) bf[p] = load_frag<T>((const char*)brow[p]);
  for (int k = 0; k < K; k += 32) {
    const int kn = k + 32 < K ? k + 32 : k;
    Frag<T> an[4], bn[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) an[c] = load_frag<T>((const char*)(arow[c] + kn));
#pragma unroll
    for (int p = 0; p < 4; ++p) bn[p] = load_frag<T>((const char*)(brow[p] + (size_t)(kn >> 6) * LS + (kn & 63)));
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int p = 0; p < 4; ++p) mfma_frag(acc[c][p], af[c], bf[p]);
#pragma unroll
    for (int c = 0; c < 4; ++c) af[c] = an[c];
#pragma unroll
    for (int p = 0; p < 4; ++p) bf[p] = bn[p];
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int co = c * 16 + 4 * g;
    float bias[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[i] = a.bias[co + i];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int n = n0 + p * 16 + (lane & 15);
      if (n >= a.N) continue;
      *(f32x4*)(a.skip + ((size_t)b * a.N + n) * DW_C + co) =
          f32x4{acc[c][p][0] + bias[0], acc[c][p][1] + bias[1], acc[c][p][2] + bias[2], acc[c][p][3] + bias[3]};
    }
  }
}

hipError_t launch_dw_skip(int dtype, const DWSkipArgs& a, hipStream_t s) {
  const dim3 grid((a.N + 255) / 256, a.B);
  if (dtype == DT_F32) hipLaunchKernelGGL(dw_skip_kernel<float>, grid, dim3(256), 0, s, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(dw_skip_kernel<bf16_t>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(dw_skip_kernel<f16_t>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------- deferred skip sum fused with the output head ----------------
// dw_skip_kernel's GEMM, then the head of dw_output_kernel straight from the accumulators: lane
// (g, l16) holds s[co = 16 c + 4 g + i][n = l16] of each tile, which is exactly the B operand of a
// 16x16x4 f32 MFMA step whose four k values are {16 c + 4 g' + i : g' = 0..3} -- so skip_projection
// consumes the skip sum from registers (16 steps per 16 outputs), and the fp32 skip rows never go
// to HBM (264 MB written and read again per step at config #3).
template <typename T>
__global__ __launch_bounds__(256) void dw_skip_head_kernel(DWSkipArgs a, DWOutArgs o) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int n0 = blockIdx.x * 256 + wave * 64, b = blockIdx.y, K = a.L * DW_C;
  const size_t LS = (size_t)a.B * a.N * DW_C;        // z is layer-major: [L][B][N][64]
  const T* Z = (const T*)a.z + (size_t)b * a.N * DW_C;
  const T* arow[4];
  const T* brow[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) arow[c] = (const T*)a.w + (size_t)(c * 16 + l16) * K + g * 8;
#pragma unroll
  for (int p = 0; p < 4; ++p) brow[p] = Z + (size_t)min(n0 + p * 16 + l16, a.N - 1) * DW_C + g * 8;
  f32x4 acc[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
  Frag<T> af[4], bf[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) af[c] = load_frag<T>((const char*)arow[c]);
#pragma unroll
  for (int p = 0; p < 4; ++p) bf[p] = load_frag<T>((const char*)brow[p]);
  for (int k = 0; k < K; k += 32) {
    const int kn = k + 32 < K ? k + 32 : k;
    Frag<T> an[4], bn[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) an[c] = load_frag<T>((const char*)(arow[c] + kn));
#pragma unroll
    for (int p = 0; p < 4; ++p) bn[p] = load_frag<T>((const char*)(brow[p] + (size_t)(kn >> 6) * LS + (kn & 63)));
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int p = 0; p < 4; ++p) mfma_frag(acc[c][p], af[c], bf[p]);
#pragma unroll
    for (int c = 0; c < 4; ++c) af[c] = an[c];
#pragma unroll
    for (int p = 0; p < 4; ++p) bf[p] = bn[p];
  }
  // skip sum / sqrt(L), as the reference divides before skip_projection
  const float rl = o.sqrt_layers;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float bias[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bias[i] = a.bias[c * 16 + 4 * g + i];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[c][p][i] = (acc[c][p][i] + bias[i]) / rl;
  }
  float part[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int oc = 0; oc < 4; ++oc) {                 // outputs 16 oc .. 16 oc + 15
    f32x4 h[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) h[p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float w = o.wsp[(oc * 16 + l16) * DW_C + c * 16 + 4 * g + i];
#pragma unroll
        for (int p = 0; p < 4; ++p) h[p] = __builtin_amdgcn_mfma_f32_16x16x4f32(w, acc[c][p][i], h[p], 0, 0, 0);
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oo = oc * 16 + 4 * g + i;
      const float bs = o.bsp[oo], wo = o.wop[oo];
#pragma unroll
      for (int p = 0; p < 4; ++p) part[p] += wo * fmaxf(h[p][i] + bs, 0.f);
    }
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    float v = part[p];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    const int n = n0 + p * 16 + l16;
    if (g == 0 && n < a.N) o.eps[(size_t)b * a.N + n] = o.bop[0] + v;
  }
}

hipError_t launch_dw_skip_head(int dtype, const DWSkipArgs& a, const DWOutArgs& o, hipStream_t s) {
  const dim3 grid((a.N + 255) / 256, a.B);
  if (dtype == DT_F32) hipLaunchKernelGGL(dw_skip_head_kernel<float>, grid, dim3(256), 0, s, a, o);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(dw_skip_head_kernel<bf16_t>, grid, dim3(256), 0, s, a, o);
  else hipLaunchKernelGGL(dw_skip_head_kernel<f16_t>, grid, dim3(256), 0, s, a, o);
  return hipGetLastError();
}

// ---------------- output: skip sum / sqrt(L) -> skip_projection -> relu -> output_projection ----------------
// diffwave.py:150-155 per sample: h = Wsp (skip / sqrt(L)) + bsp, eps = wop . relu(h) + bop.  The
// 64 x 64 skip_projection runs as fp32 MFMA (16x16x4 f32): a wave = 64 samples x all 64 outputs
// (4 x 4 tiles, K = 64 in two 32-deep fragments), B fragments = 32-byte pieces of the samples' skip
// rows scaled by 1 / sqrt(L) (as the reference divides before the projection); relu and
// output_projection from the accumulators, the 64-output sum reduced over the 4 lane groups.
__global__ __launch_bounds__(256) void dw_output_kernel(DWOutArgs a) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, l16 = lane & 15;
  const int64_t n0 = (int64_t)blockIdx.x * 256 + wave * 64;
  const float rl = a.sqrt_layers;
  f32x4 acc[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < 2; ++h) {                    // K = 64 in two 32-deep fragments
    Frag<float> af[4], bf[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) af[c] = load_frag<float>((const char*)(a.wsp + (c * 16 + l16) * DW_C + h * 32 + g * 8));
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int64_t n = min(n0 + p * 16 + l16, a.total - 1);
      bf[p] = load_frag<float>((const char*)(a.skip + n * DW_C + h * 32 + g * 8));
#pragma unroll
      for (int e = 0; e < 4; ++e) { bf[p].lo[e] = bf[p].lo[e] / rl; bf[p].hi[e] = bf[p].hi[e] / rl; }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int p = 0; p < 4; ++p) mfma_frag(acc[c][p], af[c], bf[p]);
  }
  float bs[4][4], wo[4][4];                        // this lane's 16 outputs o = 16 c + 4 g + i
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) { bs[c][i] = a.bsp[c * 16 + 4 * g + i]; wo[c][i] = a.wop[c * 16 + 4 * g + i]; }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    float part = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) part += wo[c][i] * fmaxf(acc[c][p][i] + bs[c][i], 0.f);
    part += __shfl_xor(part, 16);
    part += __shfl_xor(part, 32);
    const int64_t n = n0 + p * 16 + l16;
    if (g == 0 && n < a.total) a.eps[n] = a.bop[0] + part;
  }
}

hipError_t launch_dw_output(const DWOutArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(dw_output_kernel, dim3((unsigned)((a.total + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sddm
