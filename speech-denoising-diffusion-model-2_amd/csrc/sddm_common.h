// Common device/host helpers for the SDDM MI355X (gfx950 / CDNA4) sampler.
//
// Numerics contract:
//  * the sampler state x_t, the condition, the noise and every transition are fp32;
//  * the noise-level embedding (UNetModified2.py:49-68) is fp32 with accurate sinf/cosf;
//  * network activations are stored as T in {float, __bf16, _Float16}; MFMA accumulates fp32;
//  * GroupNorm statistics are fp32 per tile, combined in fp64 (Chan's parallel variance).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16_t;
typedef _Float16 f16_t;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

enum SddmDtype { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2 };

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 counter RNG + Box-Muller (restated in oracle/philox.py; integer part bit-exact).
// Element e of draw d: counter (lo(e>>2), hi(e>>2), d, 0x5DD3), key (lo(seed), hi(seed)).
// ---------------------------------------------------------------------------------------------
struct U32x4 { uint32_t x, y, z, w; };

__host__ __device__ __forceinline__ U32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2,
                                                         uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return U32x4{c0, c1, c2, c3};
}

__device__ __forceinline__ float philox_unit(uint32_t w) {
  return (float)((w >> 8) | 1u) * 0x1p-24f;  // exact odd 24-bit fraction in (0,1)
}

// The 4 normals of counter group q = e >> 2 (elements 4q .. 4q+3).
__device__ __forceinline__ f32x4 philox_normal4(uint64_t seed, uint32_t draw, uint64_t q) {
  const U32x4 r = philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), draw, 0x5DD3u,
                                (uint32_t)seed, (uint32_t)(seed >> 32));
  const float ra = sqrtf(-2.0f * logf(philox_unit(r.x)));
  const float rb = sqrtf(-2.0f * logf(philox_unit(r.z)));
  const float ta = 2.0f * philox_unit(r.y), tb = 2.0f * philox_unit(r.w);
  f32x4 z;
  z[0] = ra * cospif(ta); z[1] = ra * sinpif(ta);
  z[2] = rb * cospif(tb); z[3] = rb * sinpif(tb);
  return z;
}

__device__ __forceinline__ float philox_normal1(uint64_t seed, uint32_t draw, uint64_t e) {
  const f32x4 z = philox_normal4(seed, draw, e >> 2);
  return z[(int)(e & 3)];
}

// ---------------------------------------------------------------------------------------------
// Activation helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float silu(float x) { return x / (1.0f + __expf(-x)); }

template <typename T> __device__ __forceinline__ float to_f32(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v) { return (T)v; }

// fp32 clamp that propagates NaN exactly like torch.clamp_ (diffusion.py:190)
__device__ __forceinline__ float clamp_pm1(float x) {
  return x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
}

#define SDDM_HIP_CHECK(expr)                                                            \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      sddm_set_error(SDDM_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                     __FILE__, __LINE__);                                               \
      return SDDM_ERR_HIP;                                                              \
    }                                                                                   \
  } while (0)
