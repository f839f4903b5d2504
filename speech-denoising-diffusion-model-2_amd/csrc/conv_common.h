// MFMA fragment helpers shared by the convolution kernels (gfx950, wave64).
//
// 16x16 tiles with A = weights (rows = output channels) and B = pixels (cols): lane l holds
// A[co = l & 15][k = 8 (l >> 4) + j] and B[k = 8 (l >> 4) + j][px = l & 15] (j = 0..7); the fp32
// accumulator holds D[co = 4 (l >> 4) + i][px = l & 15].  For T = float the 8 channels of a
// lane group are consumed by 8 MFMA 16x16x4 instructions (element j -> k-set {j, 8+j, 16+j,
// 24+j}); any k permutation shared by A and B gives the same dot product.
#pragma once
#include <cstdlib>

#include "sddm_common.h"

namespace sddm {

template <typename T> struct Frag;
template <> struct Frag<bf16_t> { bf16x8 v; };
template <> struct Frag<f16_t> { f16x8 v; };
template <> struct Frag<float> { f32x4 lo, hi; };

template <typename T> __device__ __forceinline__ Frag<T> load_frag(const char* p);
template <> __device__ __forceinline__ Frag<bf16_t> load_frag<bf16_t>(const char* p) { return {*(const bf16x8*)p}; }
template <> __device__ __forceinline__ Frag<f16_t> load_frag<f16_t>(const char* p) { return {*(const f16x8*)p}; }
template <> __device__ __forceinline__ Frag<float> load_frag<float>(const char* p) {
  return {*(const f32x4*)p, *(const f32x4*)(p + 16)};
}

__device__ __forceinline__ void mfma_frag(f32x4& acc, const Frag<bf16_t>& a, const Frag<bf16_t>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
}
__device__ __forceinline__ void mfma_frag(f32x4& acc, const Frag<f16_t>& a, const Frag<f16_t>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a.v, b.v, acc, 0, 0, 0);
}
__device__ __forceinline__ void mfma_frag(f32x4& acc, const Frag<float>& a, const Frag<float>& b) {
#pragma unroll
  for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.lo[j], b.lo[j], acc, 0, 0, 0);
#pragma unroll
  for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.hi[j], b.hi[j], acc, 0, 0, 0);
}

template <typename T> struct Mfma {
  static __device__ __forceinline__ void run(f32x4& acc, const char* pa, const char* pb) {
    mfma_frag(acc, load_frag<T>(pa), load_frag<T>(pb));
  }
};

// GroupNorm affine + SiLU on one 16-byte vector (16 / sizeof(T) channels), re-rounded to T.
template <typename T>
__device__ __forceinline__ f32x4 transform_vec(f32x4 raw, const float* sc, const float* sh, bool gn) {
  constexpr int VE = 16 / (int)sizeof(T);
  typedef T vec __attribute__((ext_vector_type(VE)));
  if (!gn) return raw;
  vec v = __builtin_bit_cast(vec, raw);
#pragma unroll
  for (int j = 0; j < VE; ++j) v[j] = from_f32<T>(silu(to_f32<T>(v[j]) * sc[j] + sh[j]));
  return __builtin_bit_cast(f32x4, v);
}

template <typename T>
__device__ __forceinline__ void transform16(char* dst, const char* src, const float* sc, const float* sh, bool gn) {
  *(f32x4*)dst = transform_vec<T>(*(const f32x4*)src, sc, sh, gn);
}

// store 4 consecutive channels (one accumulator) as T
template <typename T> __device__ __forceinline__ void store4(T* p, float a, float b, float c, float d);
template <> __device__ __forceinline__ void store4<float>(float* p, float a, float b, float c, float d) {
  *(f32x4*)p = f32x4{a, b, c, d};
}
template <> __device__ __forceinline__ void store4<bf16_t>(bf16_t* p, float a, float b, float c, float d) {
  *(bf16x4*)p = bf16x4{(bf16_t)a, (bf16_t)b, (bf16_t)c, (bf16_t)d};
}
template <> __device__ __forceinline__ void store4<f16_t>(f16_t* p, float a, float b, float c, float d) {
  *(f16x4*)p = f16x4{(f16_t)a, (f16_t)b, (f16_t)c, (f16_t)d};
}
// the same from two packed pairs (the accumulator register pairs): one v_cvt_pk per pair
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <typename T> __device__ __forceinline__ void store4p(T* p, f32x2 a, f32x2 b) { store4<T>(p, a.x, a.y, b.x, b.y); }
template <> __device__ __forceinline__ void store4p<bf16_t>(bf16_t* p, f32x2 a, f32x2 b) {
  typedef bf16_t bf16x2_t __attribute__((ext_vector_type(2)));
  typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t x = __builtin_convertvector(a, bf16x2_t), y = __builtin_convertvector(b, bf16x2_t);
  *(u32x2_t*)p = u32x2_t{__builtin_bit_cast(unsigned int, x), __builtin_bit_cast(unsigned int, y)};
}
// bf16 / f16 / f32 pair -> two floats
template <typename T> __device__ __forceinline__ f32x2 unpack2(T a, T b) { return f32x2{to_f32<T>(a), to_f32<T>(b)}; }
template <typename T> __device__ __forceinline__ f32x4 load4(const T* p);
template <> __device__ __forceinline__ f32x4 load4<float>(const float* p) { return *(const f32x4*)p; }
template <> __device__ __forceinline__ f32x4 load4<bf16_t>(const bf16_t* p) {
  const bf16x4 v = *(const bf16x4*)p;
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
template <> __device__ __forceinline__ f32x4 load4<f16_t>(const f16_t* p) {
  const f16x4 v = *(const f16x4*)p;
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
template <typename T> __device__ __forceinline__ float round_t(float v) { return to_f32<T>(from_f32<T>(v)); }

}  // namespace sddm

namespace sddm {

// ---------------------------------------------------------------------------------------------
// GroupNorm finalize fused into a consumer's prologue (nn.GroupNorm, UNetModified2.py:117).
// Producers leave per-tile (sum, M2 about the tile mean) of every channel; the consumer block
// combines them for its image b with Chan's formula in fp64 (two deterministic passes) and
// writes per-channel scale / shift = gamma*rstd, beta - mean*gamma*rstd into LDS.
// Groups never straddle the A|B concat boundary (checked on the host).
// ---------------------------------------------------------------------------------------------
// Sum over the 16 lanes of a DPP row (lanes 16r .. 16r+15): four VALU adds with DPP operands
// (xor 1, xor 2, mirror within 8, mirror within 16), every lane of the row ends with the sum.
// __shfl_xor goes through the LDS crossbar (ds_bpermute) and a dependent chain of them costs a
// full LDS round trip per step.
template <int CTRL> __device__ __forceinline__ float dpp_f32(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_sum16(float x) {
  x += dpp_f32<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dpp_f32<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dpp_f32<0x141>(x);   // row_half_mirror
  x += dpp_f32<0x140>(x);   // row_mirror
  return x;
}

// Sum over an aligned group of tpg lanes (a power of two; tpg is block-uniform): DPP steps
// within 16 lanes, LDS-crossbar shuffles beyond
__device__ __forceinline__ float group_sum(float x, int tpg) {
  if (tpg > 1) x += dpp_f32<0xB1>(x);
  if (tpg > 2) x += dpp_f32<0x4E>(x);
  if (tpg > 4) x += dpp_f32<0x141>(x);
  if (tpg > 8) x += dpp_f32<0x140>(x);
  for (int o = 16; o < tpg; o <<= 1) x += __shfl_xor(x, o);
  return x;
}

// largest power of two <= n (n >= 1)
__device__ __forceinline__ int pow2_floor(int n) { return 1 << (31 - __builtin_clz(n)); }

struct GNFuse {
  const float* statsA; int tilesA, ntileA;
  const float* statsB; int tilesB, ntileB;
  const float* gamma; const float* beta;
  int G; float eps;
};

__device__ __forceinline__ void gn_fused_prologue(const GNFuse& f, int b, int CA, int CB, float* sc, float* sh) {
  const int C = CA + CB, cpg = C / f.G;
  const int tpg = pow2_floor(blockDim.x / f.G);   // threads per group (power of two, <= 64)
  const int g = threadIdx.x / tpg, sub = threadIdx.x - g * tpg;
  if (g >= f.G) return;
  const int c0 = g * cpg;
  const bool fromA = c0 < CA;
  const float* st = fromA ? f.statsA : f.statsB;
  const int tiles = fromA ? f.tilesA : f.tilesB;
  const int ntile = fromA ? f.ntileA : f.ntileB;
  const int Cs = fromA ? CA : CB;
  const int cs0 = fromA ? c0 : c0 - CA;
  const int items = cpg * tiles;
  const float* base = st + (size_t)b * tiles * Cs * 2;
  double s = 0.0;
  for (int i = sub; i < items; i += tpg) {
    const int c = i / tiles, t = i - c * tiles;
    s += (double)base[((size_t)t * Cs + cs0 + c) * 2];
  }
  for (int o = 1; o < tpg; o <<= 1) s += __shfl_xor(s, o);
  const double n_tot = (double)items * ntile;
  const double mean = s / n_tot;
  double m2 = 0.0;
  for (int i = sub; i < items; i += tpg) {
    const int c = i / tiles, t = i - c * tiles;
    const float* e = base + ((size_t)t * Cs + cs0 + c) * 2;
    const double d = (double)e[0] / ntile - mean;
    m2 += (double)e[1] + (double)ntile * d * d;
  }
  for (int o = 1; o < tpg; o <<= 1) m2 += __shfl_xor(m2, o);
  const double rstd = 1.0 / sqrt(m2 / n_tot + (double)f.eps);
  for (int c = sub; c < cpg; c += tpg) {
    const double scale = (double)f.gamma[c0 + c] * rstd;
    sc[c0 + c] = (float)scale;
    sh[c0 + c] = (float)((double)f.beta[c0 + c] - mean * scale);
  }
}

}  // namespace sddm

namespace sddm {
// Phase timestamps (profiling builds with -DSDDM_STAMPS only): s_memrealtime (100 MHz) of wave 0
// at block start (slot 0), at the kernel's phase boundaries (slots 1..6) and at block end (slot 7).
// The flat block index comes from the kernel (blockIdx only): gridDim would be read from the
// implicit kernel arguments by a vector load whose wait drains every load in flight.
#ifdef SDDM_STAMPS
#define SDDM_STAMP(args, k) SDDM_STAMP_AT(args, k, blockIdx.x)
#define SDDM_STAMP_AT(args, k, blk)                                                               \
  do {                                                                                            \
    if ((args).stamps && threadIdx.x == 0)                                                        \
      (args).stamps[(size_t)(blk) * 8 + (k)] = __builtin_amdgcn_s_memrealtime();                  \
  } while (0)
#else
#define SDDM_STAMP(args, k) do {} while (0)
#define SDDM_STAMP_AT(args, k, blk) do {} while (0)
#endif

#ifndef SDDM_XCD_ZIN
#define SDDM_XCD_ZIN 1   // strip and K-streamed tile blocks: channel block innermost (0: z-major, A/B builds)
#endif

// XCD-aware block order.  The logical grid (X tiles, Y images, Z channel blocks) is launched as
// one dimension; blocks are dealt round-robin over the 8 XCDs (block id % 8 shares an L2), so
// block id is mapped to position (id % 8) * total/8 + id / 8 of the z-major order: each XCD's
// blocks cover one contiguous run of channel blocks (the same weight slices) and of images and
// adjacent tiles (shared halos) and read them from its own L2 instead of each XCD fetching every
// weight slice.  Speed only, never correctness (HIP does not promise the placement).
// ZIN (channel block innermost): the channel blocks of one tile share an XCD, so the second
// block's input reads hit that XCD's L2 (layers whose weights are small next to their inputs)
template <bool ZIN = false>
__device__ __forceinline__ void xcd_block(int X, int Z, int& x, int& y, int& z) {
  if (gridDim.y > 1 || gridDim.z > 1) {             // launched in plain (x, y, z) order
    x = blockIdx.x; y = blockIdx.y; z = blockIdx.z;
    return;
  }
  const int total = (int)gridDim.x, Y = total / (X * Z);
  const int id = (int)blockIdx.x;
  const int j = (total & 7) == 0 ? (id & 7) * (total >> 3) + (id >> 3) : id;
  if (ZIN) {
    z = j % Z;
    const int r = j / Z;
    x = r % X;
    y = r / X;
    return;
  }
  x = j % X;
  const int r = j / X;
  y = r % Y;
  z = r / Y;
}

// host: the launch grid for xcd_block (SDDM_XCD=0 selects the plain order, for A/B runs)
__host__ inline dim3 xcd_grid(int X, int Y, int Z) {
  static const bool plain = std::getenv("SDDM_XCD") && std::atoi(std::getenv("SDDM_XCD")) == 0;
  return plain ? dim3(X, Y, Z) : dim3(X * Y * Z);
}

// floor(n / d) for 0 <= n < 2^21 from the float reciprocal rd = 1 / d: ((n + .5) * rd) is off by
// less than the .5 / d margin, so the truncation is exact (no integer division sequence).
__device__ __forceinline__ int fdivi(int n, float rd) { return (int)(((float)n + 0.5f) * rd); }

// GroupNorm statistics of one group loaded in a single round trip (issue() before anything waits,
// finish() after): up to GK (sum, M2) items per thread; larger producers fall back to the
// two-pass loop of gn_fused_prologue (fp64).  Chan combination in a fixed order.
template <int GK_ = 12>
struct GNLoadT {
  static constexpr int GK = GK_;
  float2 v[GK];
  float gm, bt;                 // gamma / beta of channel c0 + sub (sub < cpg), loaded with the items
  int items, tpg, sub, grp, ntile;
  bool fast;

  // `on` = false (a conv without GroupNorm) still issues the same loads, all from `safe` (any
  // readable address): the kernels call issue() unconditionally, because a load inside a branch
  // makes the compiler wait for it at the branch join, serialising this round trip in front of
  // every other load of the prologue.
  __device__ __forceinline__ void issue(const GNFuse& f, int b, int CA, int CB, bool on, const float* safe) {
    const int G = f.G > 0 ? f.G : 32;
    const int C = CA + CB, cpg = C / G;
    tpg = pow2_floor(blockDim.x / G);                 // xor butterflies: a power of two (6-wave blocks)
    grp = threadIdx.x / tpg;
    sub = threadIdx.x - grp * tpg;
    const int c0 = min(grp, G - 1) * cpg;             // threads past the last group load group G-1's
    const bool fromA = c0 < CA;
    const int tiles = max(fromA ? f.tilesA : f.tilesB, 1);
    ntile = fromA ? f.ntileA : f.ntileB;
    const int Cs = fromA ? CA : CB;
    const int cs0 = fromA ? c0 : c0 - CA;
    items = cpg * tiles;
    const float* base = on ? (fromA ? f.statsA : f.statsB) + (size_t)b * tiles * Cs * 2 : safe;
    const float rt = 1.0f / (float)tiles;
    // GK loads per thread, unconditional at clamped indices (a conditional load makes the
    // compiler drain the memory counter at the branch join); finish() ignores the items past the
    // end.  `fast` is block-uniform (the larger concat source decides).
    const int imax = cpg * (CB > 0 ? max(f.tilesA, f.tilesB) : f.tilesA);
    fast = imax <= GK * tpg;
#pragma unroll
    for (int k = 0; k < GK; ++k) {
      const int i = min(sub + k * tpg, items - 1);
      const int c = fdivi(i, rt), t = i - c * tiles;
      const int off = on ? (t * Cs + cs0 + c) * 2 : 0;   // 32-bit offsets: no 64-bit address math
      v[k] = *(const float2*)(base + off);
    }
    const int cg = on ? c0 + min(sub, cpg - 1) : 0;   // clamped: unconditional loads
    gm = (on ? f.gamma : safe)[cg];
    bt = (on ? f.beta : safe)[cg];
  }

  __device__ __forceinline__ void finish(const GNFuse& f, int b, int CA, int CB, float* sc, float* sh) {
    if (!fast) {
      gn_fused_prologue(f, b, CA, CB, sc, sh);
      return;
    }
    if (grp >= f.G) return;
    const int cpg = (CA + CB) / f.G, c0 = grp * cpg;
    // fp32 Chan combination of equal-count tiles in a fixed order (items of one thread, then
    // the xor-butterfly over the group's threads): deterministic, and accurate to ~1e-7
    // relative since only tile sums and tile-centred M2 are added
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < GK; ++k)
      if (sub + k * tpg < items) s += v[k].x;
    s = group_sum(s, tpg);
    const float n_tot = (float)items * (float)ntile;
    const float r_tot = 1.0f / n_tot, r_tile = 1.0f / (float)ntile, fn = (float)ntile;
    const float mean = s * r_tot;
    float m2 = 0.f;
#pragma unroll
    for (int k = 0; k < GK; ++k) {
      if (sub + k * tpg < items) {
        const float d = v[k].x * r_tile - mean;
        m2 += v[k].y + fn * d * d;
      }
    }
    m2 = group_sum(m2, tpg);
    const float rstd = 1.0f / sqrtf(m2 * r_tot + f.eps);
    if (sub < cpg) {
      const float scale = gm * rstd;
      sc[c0 + sub] = scale;
      sh[c0 + sub] = bt - mean * scale;
    }
    for (int c = sub + tpg; c < cpg; c += tpg) {
      const float scale = f.gamma[c0 + c] * rstd;
      sc[c0 + c] = scale;
      sh[c0 + c] = f.beta[c0 + c] - mean * scale;
    }
  }
};
using GNLoad = GNLoadT<12>;

// =============================================================================================
// Per-channel tile statistics from an fp32 LDS tile [npix][ld] (values already rounded to the
// storage type).  Writes (sum, M2 about the tile mean) for channels [0, nch).
// =============================================================================================
__device__ __forceinline__ void tile_channel_stats(const float* tile, int ld, int npix, int nch, float* dst,
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

}  // namespace sddm

namespace sddm {

// Workgroup barrier that orders LDS only.  __syncthreads() also waits for every outstanding
// global load AND store of the wave (vmcnt(0)); in an epilogue that is the full write latency of
// the stores just issued, on the critical path of the block, for nothing.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Workgroup barrier for an LDS-DMA hand-off (global_load_lds): every wave's DMA loads into LDS are
// counted by vmcnt, not lgkmcnt, so a wave must drain vmcnt before the barrier for the other
// waves to read what it loaded.  Explicit (not __syncthreads()) so that the barrier cannot be
// turned into lds_sync() by mistake and does not depend on how the fence happens to lower.
__device__ __forceinline__ void dma_sync() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ float silu_fast(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }

// SiLU of two values with packed fp32 arithmetic around the two transcendentals per value:
// y * 1 / (1 + 2^(-y log2 e))
__device__ __forceinline__ f32x2 silu2(f32x2 y) {
  const f32x2 t = y * f32x2{-1.4426950408889634f, -1.4426950408889634f};
  const f32x2 d = f32x2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)} + f32x2{1.f, 1.f};
  return y * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}

// GroupNorm affine + SiLU of one 16-byte unit (VE channels), re-rounded to T
template <typename T>
__device__ __forceinline__ f32x4 transform_regs(f32x4 raw, const float* s, const float* h) {
  constexpr int VE = 16 / (int)sizeof(T);
  typedef T vec __attribute__((ext_vector_type(VE)));
  vec v = __builtin_bit_cast(vec, raw);
#pragma unroll
  for (int j = 0; j < VE; j += 2) {
    const f32x2 x = f32x2{to_f32<T>(v[j]), to_f32<T>(v[j + 1])};
    const f32x2 o = silu2(x * f32x2{s[j], s[j + 1]} + f32x2{h[j], h[j + 1]});
    v[j] = from_f32<T>(o.x);
    v[j + 1] = from_f32<T>(o.y);
  }
  return __builtin_bit_cast(f32x4, v);
}

template <typename T>
__device__ __forceinline__ f32x4 transform_fast(f32x4 raw, const float* sc, const float* sh) {
  constexpr int VE = 16 / (int)sizeof(T);
  float s[VE], h[VE];
#pragma unroll
  for (int j = 0; j < VE; ++j) { s[j] = sc[j]; h[j] = sh[j]; }
  return transform_regs<T>(raw, s, h);
}

// GroupNorm affine + SiLU of one 16-byte unit with the per-channel scale / shift read from LDS
// as 16-byte vectors (sc, sh 16-byte aligned)
template <typename T>
__device__ __forceinline__ f32x4 transform_lds(f32x4 raw, const float* sc, const float* sh) {
  constexpr int VE = 16 / (int)sizeof(T);
  float s[VE], h[VE];
#pragma unroll
  for (int j = 0; j < VE; j += 4) {
    const f32x4 a = *(const f32x4*)(sc + j), c = *(const f32x4*)(sh + j);
#pragma unroll
    for (int i = 0; i < 4; ++i) { s[j + i] = a[i]; h[j + i] = c[i]; }
  }
  return transform_regs<T>(raw, s, h);
}

// an MFMA operand fragment whose 16-byte units sit in consecutive planes `stride` bytes apart
template <typename T> __device__ __forceinline__ Frag<T> load_planes(const char* p, int stride);
template <> __device__ __forceinline__ Frag<bf16_t> load_planes<bf16_t>(const char* p, int) { return {*(const bf16x8*)p}; }
template <> __device__ __forceinline__ Frag<f16_t> load_planes<f16_t>(const char* p, int) { return {*(const f16x8*)p}; }
template <> __device__ __forceinline__ Frag<float> load_planes<float>(const char* p, int stride) {
  return {*(const f32x4*)p, *(const f32x4*)(p + stride)};
}

}  // namespace sddm
