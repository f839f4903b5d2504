// WaveGrad denoiser (reference model/wavegrad.py) for SDDM_spectrogram.infer (model.py:212-257).
//
// Activations are sample-major [B][T][C] in the compute dtype, so one time position's channels
// are contiguous and each MFMA operand fragment (8 channels) is one 16-byte (bf16/f16) or two
// 16-byte (fp32) vector loads.  Every convolution of the network -- DBlock / UBlock dilated convs,
// the 1x1 residual_dense / block1, FiLM input/output convs, first_conv and last_conv -- is one
// launch of wg_conv_kernel: an implicit GEMM over K = taps x Cin whose B-operand loader applies
// the layer's input transform on the fly (nearest up/down interpolation as an index map, the
// leaky_relu, the FiLM affine shift + scale * x) and whose epilogue fuses bias, the FiLM
// input_conv's leaky_relu + PositionalEncoding, and the residual adds.  Nothing but conv outputs
// is ever written to HBM.
//
// Block = 4 waves (256 threads) = 64 output channels x 128 time positions; wave w owns output
// channels [32 (w & 1), +32) x time [64 (w >> 1), +64) as 2 x 4 MFMA 16x16 tiles.
#include "conv_common.h"
#include "wg_kernels.h"

#include <cstdlib>

namespace sddm {

constexpr int WG_MC = 64;    // output channels per block
constexpr int WG_MT = 128;   // time positions per block

__device__ __forceinline__ float wg_leaky(float x) { return x > 0.f ? x : x * 0.2f; }

template <typename T> __device__ __forceinline__ void load8(const T* p, float* v);
template <> __device__ __forceinline__ void load8<float>(const float* p, float* v) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { v[j] = a[j]; v[4 + j] = b[j]; }
}
template <> __device__ __forceinline__ void load8<bf16_t>(const bf16_t* p, float* v) {
  const bf16x8 a = *(const bf16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)a[j];
}
template <> __device__ __forceinline__ void load8<f16_t>(const f16_t* p, float* v) {
  const f16x8 a = *(const f16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (float)a[j];
}

template <typename T> __device__ __forceinline__ Frag<T> pack8(const float* v);
template <> __device__ __forceinline__ Frag<float> pack8<float>(const float* v) {
  return {f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}};
}
template <> __device__ __forceinline__ Frag<bf16_t> pack8<bf16_t>(const float* v) {
  bf16x8 a;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = (bf16_t)v[j];
  return {a};
}
template <> __device__ __forceinline__ Frag<f16_t> pack8<f16_t>(const float* v) {
  f16x8 a;
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = (f16_t)v[j];
  return {a};
}

template <typename T> __device__ __forceinline__ Frag<T> zero_frag() {
  float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  return pack8<T>(z);
}

// t / f through the float reciprocal instead of an integer division sequence per staged element
// (the reciprocal of the uniform f is hoisted): fdivi is exact for 0 <= t < 2^21, and one
// correction step each way keeps the quotient exact while the float estimate is off by at most
// one, i.e. for every t < 2^23 (launch_wg_conv rejects longer signals)
__device__ __forceinline__ int wg_map(int t, int map, int f) {
  if (map != WG_MAP_UP) return map == WG_MAP_DOWN ? t * f : t;
  int q = fdivi(t, 1.0f / (float)f);
  q -= q * f > t ? 1 : 0;
  q += (q + 1) * f <= t ? 1 : 0;
  return q;
}

// epilogue FiLM of the next conv's input (wavegrad.py:98-99, 104-105, 107-108): m = leaky(shift +
// scale * v) for 4 channels at output element o; fp (shift) and fp + Cout (scale) at the same
// position.  Moving the modulation here reads shift / scale once per element instead of once per
// output-channel block of the consuming conv, and the consumer stages a plain input
template <typename T>
__device__ __forceinline__ void wg_film_epilogue(const WGConvArgs& a, const T* fp, size_t o, const float* v) {
#pragma clang fp contract(off)
  const f32x4 sh = load4<T>(fp), sc = load4<T>(fp + a.Cout);
  float m[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) m[e] = wg_leaky(sh[e] + sc[e] * v[e]);
  if (a.post_film == 2) {
    store4<T>((T*)a.out + o, v[0], v[1], v[2], v[3]);
    store4<T>((T*)a.out2 + o, m[0], m[1], m[2], m[3]);
  } else {
    store4<T>((T*)a.out + o, m[0], m[1], m[2], m[3]);
  }
}

// B fragment at conv-input position tp (already bounds-checked by the caller via ok)
template <typename T, int PRE>
__device__ __forceinline__ Frag<T> wg_load_b(const WGConvArgs& a, const T* src_b, const T* film_b, int tp, bool ok,
                                             int ci) {
#pragma clang fp contract(off)
  if (!ok) return zero_frag<T>();
  const int sr = wg_map(tp, a.map, a.f);
  const T* p = src_b + (size_t)sr * a.src_C + ci;
  if (PRE == 0) return load_frag<T>((const char*)p);
  float v[8];
  load8<T>(p, v);
  if (PRE == 2) {            // leaky(shift + scale * x)   (wavegrad.py:98, 104, 107)
    float sh[8], sc[8];
    const T* fp = film_b + (size_t)tp * 2 * a.Cin + ci;
    load8<T>(fp, sh);
    load8<T>(fp + a.Cin, sc);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = wg_leaky(sh[j] + sc[j] * v[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = wg_leaky(v[j]);
  }
  return pack8<T>(v);
}

template <typename T, int PRE>
__global__ __launch_bounds__(256) void wg_conv_kernel(WGConvArgs a) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, l16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.z;
  const int co0 = blockIdx.y * WG_MC + (wave & 1) * 32;
  const int tt0 = blockIdx.x * WG_MT + (wave >> 1) * 64;
  const int Tc = a.Tc, Cin = a.Cin, KC = a.K * Cin, half = (a.K - 1) / 2;
  const T* src_b = (const T*)a.src + (size_t)b * a.src_T * a.src_C;
  const T* film_b = PRE == 2 ? (const T*)a.film + (size_t)b * Tc * 2 * Cin : nullptr;
  const T* wrow[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) wrow[c] = (const T*)a.w + (size_t)(co0 + c * 16 + l16) * KC + g * 8;

  f32x4 acc[2][4];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[c][p] = f32x4{0.f, 0.f, 0.f, 0.f};

  // flattened K loop over (tap, 32-channel chunk), operands of step s + 1 loaded before the
  // MFMAs of step s (register double buffer: the loads' latency hides behind 8 MFMAs per wave)
  const int ncs = Cin / 32, nsteps = a.K * ncs;
  auto load_step = [&](int st, Frag<T>* af, Frag<T>* bfr) {
    const int tap = st / ncs, c0 = (st - tap * ncs) * 32;
#pragma unroll
    for (int c = 0; c < 2; ++c) af[c] = load_frag<T>((const char*)(wrow[c] + tap * Cin + c0));
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int t = tt0 + p * 16 + l16;
      const int tp = t + (tap - half) * a.dil;
      const bool ok = t < Tc && tp >= 0 && tp < Tc;
      bfr[p] = wg_load_b<T, PRE>(a, src_b, film_b, tp, ok, c0 + g * 8);
    }
  };
  Frag<T> af[2], bfr[4];
  load_step(0, af, bfr);
  for (int st = 0; st < nsteps; ++st) {
    Frag<T> an[2], bn[4];
    if (st + 1 < nsteps) load_step(st + 1, an, bn);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int p = 0; p < 4; ++p) mfma_frag(acc[c][p], af[c], bfr[p]);
    if (st + 1 < nsteps) {
#pragma unroll
      for (int c = 0; c < 2; ++c) af[c] = an[c];
#pragma unroll
      for (int p = 0; p < 4; ++p) bfr[p] = bn[p];
    }
  }

  // epilogue: bias, FiLM leaky + encoding, residual, store
  const float* enc = nullptr;
  if (a.post == 1) {
    const int row = a.enc_per_b ? b : *a.t_dev;
    enc = a.enc + (size_t)row * a.enc_stride + a.enc_off;
  }
  const T* res_b = a.res ? (const T*)a.res + (size_t)b * a.res_T * a.Cout : nullptr;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int cb = co0 + c * 16 + 4 * g;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int t = tt0 + p * 16 + l16;
      if (t >= Tc) continue;
      float v[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int co = cb + i;
        float x = acc[c][p][i] + (co < a.Cout ? a.bias[co] : 0.f);
        if (a.post == 1 && co < a.Cout) x = wg_leaky(x) + enc[co];
        if (res_b && co < a.Cout) x = x + to_f32<T>(res_b[(size_t)wg_map(t, a.res_map, a.res_f) * a.Cout + co]);
        v[i] = x;
      }
      if (a.out_f32) {
        float* o = (float*)a.out + ((size_t)b * Tc + t) * a.Cout;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (cb + i < a.Cout) o[cb + i] = v[i];
      } else if ((a.Cout & 3) == 0) {
        const size_t o = ((size_t)b * Tc + t) * a.Cout + cb;
        if (cb < a.Cout && a.post_film)
          wg_film_epilogue<T>(a, (const T*)a.efilm + ((size_t)b * Tc + t) * 2 * a.Cout + cb, o, v);
        else if (cb < a.Cout) store4<T>((T*)a.out + o, v[0], v[1], v[2], v[3]);
      } else {
        T* o = (T*)a.out + ((size_t)b * Tc + t) * a.Cout;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (cb + i < a.Cout) o[cb + i] = from_f32<T>(v[i]);
      }
    }
  }
}

// ---------------- LDS-staged variant for Cout % 128 == 0 ----------------
// Block = 4 waves = 128 output channels x 128 positions; wave w owns channels [64 (w & 1), +64) x
// positions [64 (w >> 1), +64) as 4 x 4 MFMA tiles.  Per 32-channel chunk of the input the block
// stages (a) the transformed input slab of 128 + 2 * halo rows once (index map, zero padding and
// leaky applied here, once per element) and (b) the weights of all KT taps for its 128 channels;
// every tap then reads its B fragments from the slab at a row offset of tap * dil.  The next
// chunk's global loads are issued before the current chunk's MFMAs.
constexpr int WGL_MC = 128, WGL_HALO = 8;

// TW = waves along time: block = 2 x TW waves = 128 channels x 64 TW positions (TW = 4 halves the
// per-position weight traffic from L2 on the long levels).  The 3-tap variants without FiLM are
// held to 168 registers (three waves per SIMD, three blocks per CU: 135 vs 148 and 103 vs 114 us
// per launch); the FiLM variant spills there (364 vs 252 us) and the 1-tap ones gain nothing.
// WD: the weight image of each chunk goes global -> LDS by DMA (global_load_lds, no staging
// registers), single-buffered: issued after the barrier that frees the image, waited before the
// chunk's MFMAs; with WD the FiLM variant is held to three blocks per CU
template <typename T, int PRE, int KT, int TW, int WD = 0>
__global__ __launch_bounds__(128 * TW, (TW == 2 && KT == 3 && (PRE != 2 || WD)) ? 3 : 2) void wg_conv_lds_kernel(WGConvArgs a) {
#pragma clang fp contract(off)
  constexpr int NT = 128 * TW, WGL_MT = 64 * TW;
  constexpr int ES = (int)sizeof(T), UE = 16 / ES;         // elements per 16-byte unit
  constexpr int UPR = 32 / UE;                              // units per 32-channel row
  constexpr int RS = UPR * 16 + 16;                         // padded LDS row stride (bytes)
  constexpr int SROWS = WGL_MT + 2 * WGL_HALO;
  constexpr int NBU = SROWS * UPR, NAU = KT * WGL_MC * UPR;
  constexpr int PB = (NBU + NT - 1) / NT, PA = WD ? 1 : (NAU + NT - 1) / NT;
  static_assert(!WD || (ES == 2 && (KT * WGL_MC) % 64 == 0), "weight DMA: 16-bit, whole 64-slot runs");
  // 16-bit storage: plane-major images (a plane = one 16-byte channel unit of every row, plane
  // stride 0 mod 256 B) with the row slot XOR-swizzled by 2 x plane, so the staging stores (8-lane
  // groups: 2 rows x 4 planes) and the MFMA operand reads (ds_read_b128 lane groups mixing 8 rows
  // of two planes) hit distinct banks; fp32 keeps the padded row-major image
  constexpr bool SW = ES == 2;
  constexpr int PSB = (SROWS * 16 + 255) / 256 * 256, PSW = (KT * WGL_MC * 16 + 255) / 256 * 256;
  constexpr int SLAB_BYTES = SW ? UPR * PSB : SROWS * RS, WL_BYTES = SW ? UPR * PSW : KT * WGL_MC * RS;
  static_assert(!SW || (SROWS % 8 == 0 && UPR <= 4), "the swizzle stays inside aligned 8-row groups");
  __shared__ __attribute__((aligned(16))) char lds[SLAB_BYTES + WL_BYTES];
  char* slab = lds;
  char* wl = lds + SLAB_BYTES;
  auto sadr = [](int r, int q) { return SW ? q * PSB + ((r ^ (q << 1)) << 4) : r * RS + q * 16; };
  auto wadr = [](int r, int q) { return SW ? q * PSW + ((r ^ (q << 1)) << 4) : r * RS + q * 16; };

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, l16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int b = blockIdx.z, cob = blockIdx.y * WGL_MC, t0 = blockIdx.x * WGL_MT;
  const int Tc = a.Tc, Cin = a.Cin, half = (KT - 1) / 2, H = half * a.dil;
  const int rows = WGL_MT + 2 * H;
  const T* src_b = (const T*)a.src + (size_t)b * a.src_T * a.src_C;
  const T* W = (const T*)a.w;

  constexpr int PF = PRE == 2 ? PB : 1;
  f32x4 breg[PB], areg[PA], shreg[PF], screg[PF];
  const T* film_b = PRE == 2 ? (const T*)a.film + (size_t)b * Tc * 2 * Cin : nullptr;
  auto gload = [&](int c0) {
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int u = tid + j * NT;
      const int r = u / UPR, q = u - r * UPR;
      const int tp = t0 - H + r;
      breg[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const bool in = u < rows * UPR && tp >= 0 && tp < Tc;
      if (in) breg[j] = *(const f32x4*)(src_b + (size_t)wg_map(tp, a.map, a.f) * a.src_C + c0 + q * UE);
      if (PRE == 2 && in) {               // FiLM shift / scale at the conv-input position
        const T* fp = film_b + (size_t)tp * 2 * Cin + c0 + q * UE;
        shreg[j % PF] = *(const f32x4*)fp;
        screg[j % PF] = *(const f32x4*)(fp + Cin);
      }
    }
    if (!WD) {
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const int u = tid + j * NT;
        const int k = u / (WGL_MC * UPR), rem = u - k * (WGL_MC * UPR), co = rem / UPR, q = rem - co * UPR;
        if (u < NAU) areg[j] = *(const f32x4*)(W + ((size_t)(cob + co) * KT + k) * Cin + c0 + q * UE);
      }
    }
  };
  // weight image of chunk c0 by DMA: plane q holds KT * 128 slots in 64-slot runs, one run per wave
  // instruction; lane l of a run starting at slot s0 fetches row r = (s0 + l) ^ 2q (the swizzle)
  auto wdma = [&](int c0) {
    constexpr int RUNS = UPR * KT * WGL_MC / 64, RPW = (RUNS + NT / 64 - 1) / (NT / 64);
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const int run = wave * RPW + i;                  // wave-uniform
      if (run < RUNS) {
        const int q = run / (KT * WGL_MC / 64), s0 = (run - q * (KT * WGL_MC / 64)) * 64;
        const int r = (s0 + lane) ^ (q << 1), k = r / WGL_MC, co = r - k * WGL_MC;
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(W + ((size_t)(cob + co) * KT + k) * Cin + c0 + q * UE),
            (__attribute__((address_space(3))) void*)(wl + q * PSW + s0 * 16), 16, 0, 0);
      }
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int u = tid + j * NT;
      if (u >= rows * UPR) continue;
      const int r = u / UPR, q = u - r * UPR;
      f32x4 v = breg[j];
      const int tp = t0 - H + r;
      if (PRE == 1) {
        typedef T vec __attribute__((ext_vector_type(UE)));
        vec x = __builtin_bit_cast(vec, v);
#pragma unroll
        for (int e = 0; e < UE; ++e) x[e] = from_f32<T>(wg_leaky(to_f32<T>(x[e])));
        v = __builtin_bit_cast(f32x4, x);
      } else if (PRE == 2 && tp >= 0 && tp < Tc) {   // leaky(shift + scale * x); padding stays 0
        typedef T vec __attribute__((ext_vector_type(UE)));
        vec x = __builtin_bit_cast(vec, v);
        const vec sh = __builtin_bit_cast(vec, shreg[j % PF]), sc = __builtin_bit_cast(vec, screg[j % PF]);
#pragma unroll
        for (int e = 0; e < UE; ++e) x[e] = from_f32<T>(wg_leaky(to_f32<T>(sh[e]) + to_f32<T>(sc[e]) * to_f32<T>(x[e])));
        v = __builtin_bit_cast(f32x4, x);
      }
      *(f32x4*)(slab + sadr(r, q)) = v;
    }
    if (!WD) {
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const int u = tid + j * NT;
        if (u >= NAU) continue;
        const int k = u / (WGL_MC * UPR), rem = u - k * (WGL_MC * UPR), co = rem / UPR, q = rem - co * UPR;
        *(f32x4*)(wl + wadr(k * WGL_MC + co, q)) = areg[j];
      }
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int p = 0; p < 4; ++p) acc[i][p] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wc = (wave & 1) * 64, wt = (wave >> 1) * 64;
  const int wa0 = SW ? wadr(wc + l16, g) : 0;
  const int ncs = Cin / 32;
  gload(0);
  for (int cc = 0; cc < ncs; ++cc) {
    __syncthreads();
    if (WD) wdma(cc * 32);
    lstore();
    if (WD) dma_sync();                                  // the weight DMAs landed, the slab stored
    else __syncthreads();
    if (cc + 1 < ncs) gload((cc + 1) * 32);
#pragma unroll
    for (int k = 0; k < KT; ++k) {
      Frag<T> af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)   // (rows k * 128 + i * 16 keep the swizzled low bits: constant offsets)
        af[i] = load_frag<T>(wl + (SW ? wa0 + (k * WGL_MC + i * 16) * 16 : (k * WGL_MC + wc + i * 16 + l16) * RS + g * 8 * ES));
      const int sbk = SW ? sadr(wt + l16 + k * a.dil, g) : 0;
#pragma unroll
      for (int p = 0; p < 4; ++p)
        bf[p] = load_frag<T>(slab + (SW ? sbk + p * 16 * 16 : (wt + p * 16 + l16 + k * a.dil) * RS + g * 8 * ES));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int p = 0; p < 4; ++p) mfma_frag(acc[i][p], af[i], bf[p]);
    }
  }

  const float* enc = nullptr;
  if (a.post == 1) {
    const int row = a.enc_per_b ? b : *a.t_dev;
    enc = a.enc + (size_t)row * a.enc_stride + a.enc_off;
  }
  const T* res_b = a.res ? (const T*)a.res + (size_t)b * a.res_T * a.Cout : nullptr;
  const T* ef_b = a.post_film ? (const T*)a.efilm + (size_t)b * Tc * 2 * a.Cout : nullptr;
  // FiLM operands (shift, scale) of the epilogue: 16-bit storage loads all 16 tiles' at once (64
  // VGPRs, free once the K loop is done), so a block waits on them once; fp32 loads them per
  // channel group.  Positions are clamped (rows past Tc are not stored)
  typedef T vec4 __attribute__((ext_vector_type(4)));
  constexpr int GI = sizeof(T) == 2 ? 4 : 1;
  vec4 sh[GI][4], sc[GI][4];
  if (GI == 4 && ef_b) {
#pragma unroll
    for (int i = 0; i < GI; ++i)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const T* fp = ef_b + (size_t)min(t0 + wt + p * 16 + l16, Tc - 1) * 2 * a.Cout + cob + wc + i * 16 + 4 * g;
        sh[i][p] = *(const vec4*)fp;
        sc[i][p] = *(const vec4*)(fp + a.Cout);
      }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cb = cob + wc + i * 16 + 4 * g;
    const int fi = GI == 4 ? i : 0;
    float bias[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[e] = a.bias[cb + e];
    // the residual operands of the 4 position tiles are loaded together, so a channel group waits
    // on memory once rather than once per tile
    vec4 rv[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int tcl = min(t0 + wt + p * 16 + l16, Tc - 1);
      if (res_b) rv[p] = *(const vec4*)(res_b + (size_t)wg_map(tcl, a.res_map, a.res_f) * a.Cout + cb);
      if (GI == 1 && ef_b) {
        sh[0][p] = *(const vec4*)(ef_b + (size_t)tcl * 2 * a.Cout + cb);
        sc[0][p] = *(const vec4*)(ef_b + (size_t)tcl * 2 * a.Cout + a.Cout + cb);
      }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int t = t0 + wt + p * 16 + l16;
      if (t >= Tc) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = acc[i][p][e] + bias[e];
        if (a.post == 1) x = wg_leaky(x) + enc[cb + e];
        if (res_b) x = x + to_f32<T>(rv[p][e]);
        v[e] = x;
      }
      const size_t o = ((size_t)b * Tc + t) * a.Cout + cb;
      if (ef_b) {
        float m[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) m[e] = wg_leaky(to_f32<T>(sh[fi][p][e]) + to_f32<T>(sc[fi][p][e]) * v[e]);
        if (a.post_film == 2) store4<T>((T*)a.out2 + o, m[0], m[1], m[2], m[3]);
        else { v[0] = m[0]; v[1] = m[1]; v[2] = m[2]; v[3] = m[3]; }
      }
      store4<T>((T*)a.out + o, v[0], v[1], v[2], v[3]);
    }
  }
}

bool wg_conv_uses_lds(const WGConvArgs& a) {
  static const bool off = std::getenv("SDDM_WG_NO_LDS") != nullptr;
  return !off && a.Cout % WGL_MC == 0 && !a.out_f32 && (a.K == 3 && a.dil <= WGL_HALO) ||
         (!off && a.Cout % WGL_MC == 0 && !a.out_f32 && a.K == 1 && a.pre != 2);
}

template <typename T, int PRE, int TW>
static void wg_conv_lds_dispatch(const WGConvArgs& a, hipStream_t s) {
  const dim3 grid((a.Tc + 64 * TW - 1) / (64 * TW), a.Cout / WGL_MC, a.B);
  static const bool wd = std::getenv("SDDM_WG_FILM_DMA") != nullptr;   // experiment knob
  if (a.K == 1) hipLaunchKernelGGL((wg_conv_lds_kernel<T, PRE == 2 ? 0 : PRE, 1, TW>), grid, dim3(128 * TW), 0, s, a);
  else if (PRE == 2 && TW == 2 && sizeof(T) == 2 && wd)
    hipLaunchKernelGGL((wg_conv_lds_kernel<T, PRE, 3, TW, sizeof(T) == 2 ? 1 : 0>), grid, dim3(128 * TW), 0, s, a);
  else hipLaunchKernelGGL((wg_conv_lds_kernel<T, PRE, 3, TW>), grid, dim3(128 * TW), 0, s, a);
}

template <typename T, int PRE>
static void wg_conv_lds_pick(const WGConvArgs& a, hipStream_t s) {
  static const int tw_env = std::getenv("SDDM_WG_TW") ? std::atoi(std::getenv("SDDM_WG_TW")) : 0;
  const bool wide = tw_env == 4;   // 256-position tiles: measured no faster (165 vs 169 audio-s/s)
  if (wide) wg_conv_lds_dispatch<T, PRE, 4>(a, s);
  else wg_conv_lds_dispatch<T, PRE, 2>(a, s);
}

// last_conv (Conv1d(128, 1, 3, padding=1), wavegrad.py:164, 178): an MFMA tile would be 1/128
// useful, so each 16-lane group reads one position's 128 channels as 16 contiguous 16-byte units
// (coalesced), forms the three tap dot products d_k[p] = w_k . x[p] with a 16-lane shuffle
// reduction, parks them in LDS, and out[t] = bias + d_0[t-1] + d_1[t] + d_2[t+1].
constexpr int WG1_MT = 128;
template <typename T>
__global__ __launch_bounds__(256) void wg_last_kernel(WGConvArgs a) {
#pragma clang fp contract(off)
  __shared__ float d[3][WG1_MT + 2];
  const int tid = threadIdx.x, grp = tid >> 4, l = tid & 15;
  const int b = blockIdx.y, t0 = blockIdx.x * WG1_MT, Tc = a.Tc;
  const T* src_b = (const T*)a.src + (size_t)b * a.src_T * a.src_C;
  float w[3][8];
#pragma unroll
  for (int k = 0; k < 3; ++k) load8<T>((const T*)a.w + k * 128 + l * 8, w[k]);
  for (int r = grp; r < WG1_MT + 2; r += 16) {      // positions t0 - 1 .. t0 + WG1_MT
    const int p = t0 - 1 + r;
    float acc[3] = {0.f, 0.f, 0.f};
    if (p >= 0 && p < Tc) {
      float v[8];
      load8<T>(src_b + (size_t)p * a.src_C + l * 8, v);
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[k] += w[k][e] * v[e];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) acc[k] += __shfl_xor(acc[k], o, 16);
    if (l == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) d[k][r] = acc[k];
    }
  }
  __syncthreads();
  if (tid < WG1_MT) {
    const int t = t0 + tid;
    if (t < Tc) ((float*)a.out)[(size_t)b * Tc + t] = a.bias[0] + d[0][tid] + d[1][tid + 1] + d[2][tid + 2];
  }
}

template <typename T>
static void wg_conv_dispatch(const WGConvArgs& a, dim3 grid, hipStream_t s) {
  static const bool no_last = std::getenv("SDDM_WG_NO_LAST") != nullptr;
  if (!no_last && a.Cout == 1 && a.out_f32 && a.K == 3 && a.dil == 1 && a.Cin == 128 && a.pre == 0 &&
      a.map == WG_MAP_ID && !a.res && a.post == 0) {
    hipLaunchKernelGGL(wg_last_kernel<T>, dim3((a.Tc + WG1_MT - 1) / WG1_MT, a.B), dim3(256), 0, s, a);
    return;
  }
  if (wg_conv_uses_lds(a)) {
    if (a.pre == 0) wg_conv_lds_pick<T, 0>(a, s);
    else if (a.pre == 1) wg_conv_lds_pick<T, 1>(a, s);
    else wg_conv_lds_pick<T, 2>(a, s);
    return;
  }
  if (a.pre == 0) hipLaunchKernelGGL((wg_conv_kernel<T, 0>), grid, dim3(256), 0, s, a);
  else if (a.pre == 1) hipLaunchKernelGGL((wg_conv_kernel<T, 1>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((wg_conv_kernel<T, 2>), grid, dim3(256), 0, s, a);
}

hipError_t launch_wg_conv(int dtype, const WGConvArgs& a, hipStream_t s) {
  if (a.Cin % 32 || a.Cin > a.src_C || a.K < 1 || a.K % 2 == 0 || a.Tc < 1 || a.B < 1 || a.Cout < 1)
    return hipErrorInvalidValue;
  if ((a.map == WG_MAP_UP && (a.f < 1 || a.src_T * a.f != a.Tc)) || (a.map == WG_MAP_DOWN && a.src_T / a.f != a.Tc) ||
      (a.map == WG_MAP_ID && a.src_T != a.Tc) || (a.pre == 2 && !a.film) || (a.post == 1 && (!a.enc || (!a.enc_per_b && !a.t_dev))))
    return hipErrorInvalidValue;
  if (a.post_film && (a.post_film > 2 || !a.efilm || a.out_f32 || a.Cout % 4 || (a.post_film == 2 && !a.out2)))
    return hipErrorInvalidValue;
  if (a.res && ((a.res_map == WG_MAP_UP && a.res_T * a.res_f != a.Tc) || (a.res_map == WG_MAP_ID && a.res_T != a.Tc)))
    return hipErrorInvalidValue;
  if (a.Tc >= kWgMaxPositions || a.src_T >= kWgMaxPositions)   // wg_map's exact range
    return hipErrorInvalidValue;
  const dim3 grid((a.Tc + WG_MT - 1) / WG_MT, (a.Cout + WG_MC - 1) / WG_MC, a.B);
  if (dtype == DT_F32) wg_conv_dispatch<float>(a, grid, s);
  else if (dtype == DT_BF16) wg_conv_dispatch<bf16_t>(a, grid, s);
  else wg_conv_dispatch<f16_t>(a, grid, s);
  return hipGetLastError();
}

// ---------------- downsample.0: Conv1d(1, 32, 5, padding=2) ----------------
template <typename T>
__global__ __launch_bounds__(256) void wg_first_kernel(WGFirstArgs a) {
  __shared__ float w[32 * 5], bias[32];
  const int tid = threadIdx.x;
  if (a.t_dev && blockIdx.x == 0 && tid == 0) *a.t_dev -= 1;   // this step's t
  if (tid < 160) w[tid] = a.w[tid];
  if (tid < 32) bias[tid] = a.b[tid];
  __syncthreads();
  const int64_t total = (int64_t)a.B * a.N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + tid; i < total; i += (int64_t)gridDim.x * 256) {
    const int n = (int)(i % a.N);
    const float* x = a.audio + (i - n);
    float xv[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int m = n + k - 2;
      xv[k] = (m >= 0 && m < a.N) ? x[m] : 0.f;
    }
    T* o = (T*)a.out + i * 32;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = q * 4 + e;
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < 5; ++k) s += w[co * 5 + k] * xv[k];
        v[e] = s + bias[co];
      }
      store4<T>(o + q * 4, v[0], v[1], v[2], v[3]);
    }
  }
}

hipError_t launch_wg_first(int dtype, const WGFirstArgs& a, hipStream_t s) {
  const int64_t total = (int64_t)a.B * a.N;
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 16384)));
  if (dtype == DT_F32) hipLaunchKernelGGL(wg_first_kernel<float>, grid, dim3(256), 0, s, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(wg_first_kernel<bf16_t>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(wg_first_kernel<f16_t>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------- FiLM modulation + leaky_relu (one pass, 8 channels per thread) ----------------
template <typename T>
__global__ __launch_bounds__(256) void wg_film_kernel(WGFilmArgs a) {
#pragma clang fp contract(off)
  const int cv = a.C / 8;
  const int64_t total = a.BT * cv;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t bt = i / cv;
    const int c = (int)(i - bt * cv) * 8;
    float x[8], sh[8], sc[8];
    load8<T>((const T*)a.x + bt * a.C + c, x);
    load8<T>((const T*)a.film + bt * 2 * a.C + c, sh);
    load8<T>((const T*)a.film + bt * 2 * a.C + a.C + c, sc);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = wg_leaky(sh[j] + sc[j] * x[j]);
    const Frag<T> f = pack8<T>(x);
    *(Frag<T>*)((T*)a.out + bt * a.C + c) = f;
  }
}

hipError_t launch_wg_film(int dtype, const WGFilmArgs& a, hipStream_t s) {
  if (a.C % 8) return hipErrorInvalidValue;
  const int64_t total = a.BT * (a.C / 8);
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 32768)));
  if (dtype == DT_F32) hipLaunchKernelGGL(wg_film_kernel<float>, grid, dim3(256), 0, s, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(wg_film_kernel<bf16_t>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(wg_film_kernel<f16_t>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------- spectrogram [B][C][F] -> [B][F][C] ----------------
template <typename T>
__global__ __launch_bounds__(256) void wg_spec_kernel(WGSpecArgs a) {
  const int64_t total = (int64_t)a.B * a.F * a.C;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int c = (int)(i % a.C);
    const int64_t bf = i / a.C;
    const int f = (int)(bf % a.F), b = (int)(bf / a.F);
    ((T*)a.out)[i] = from_f32<T>(a.spec[((size_t)b * a.C + c) * a.F + f]);
  }
}

hipError_t launch_wg_spec(int dtype, const WGSpecArgs& a, hipStream_t s) {
  const int64_t total = (int64_t)a.B * a.F * a.C;
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 16384)));
  if (dtype == DT_F32) hipLaunchKernelGGL(wg_spec_kernel<float>, grid, dim3(256), 0, s, a);
  else if (dtype == DT_BF16) hipLaunchKernelGGL(wg_spec_kernel<bf16_t>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(wg_spec_kernel<f16_t>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// ---------------- PositionalEncoding rows (wavegrad.py:44-49) ----------------
__global__ __launch_bounds__(256) void wg_enc_kernel(WGEncArgs a) {
#pragma clang fp contract(off)
  const int r = blockIdx.x;
  const float nl = a.noise_levels ? a.noise_levels[r] : (a.time_step_mode ? (float)r : a.table[r]);
  for (int j = threadIdx.x; j < a.n; j += 256) {
    int i = 0;
#pragma unroll
    for (int q = 1; q < 5; ++q)
      if (j >= a.offs[q]) i = q;
    const int k = j - a.offs[i], cnt = a.dims[i] / 2;
    const float e = nl * a.ev[a.offs[i] / 2 + (k % cnt)];
    a.out[(size_t)r * a.stride + j] = k < cnt ? sinf(e) : cosf(e);
  }
}

hipError_t launch_wg_enc(const WGEncArgs& a, hipStream_t s) {
  if (a.R < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(wg_enc_kernel, dim3(a.R), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sddm
