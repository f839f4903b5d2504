// Forward-process noising (q_sample) of the reference's training step, model/diffusion.py:225-279.
// One elementwise pass over [B][N]; the per-row noise level is derived from the caller's t / r
// (drawn with torch's generator by the facade, as the reference does) in the reference's
// operation order with FP contraction off.
#include "q_kernels.h"

namespace sddm {

__global__ __launch_bounds__(256) void q_sample_kernel(QArgs a) {
#pragma clang fp contract(off)
  const int64_t total = a.B * a.N;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / a.N;
    const int64_t t = a.t[b];
    const float x0 = a.x0[i], z = a.noise[i];
    if (a.mode == 0) {
      float s;
      if (a.r) {
        const float la = a.sab[t - 1], lb = a.sab[t], r = a.r[b];
        s = la + r * (lb - la);
      } else {
        s = a.sab[t];
      }
      a.x_t[i] = s * x0 + sqrtf(1.f - s * s) * z;
      if (i % a.N == 0) {
        if (a.s_out) a.s_out[b] = s;
        if (a.level_out) a.level_out[b] = (float)t + (a.r ? a.r[b] : 0.f);
      }
    } else {
      const float sab = a.sab[t];
      const float g = a.sqrt_delta[t] * z;
      const float c = a.m[t] * sab * (a.y[i] - x0);
      a.x_t[i] = sab * x0 + c + g;
      if (a.combined) a.combined[i] = 1.f / sqrtf(1.f - a.alpha_bar[t]) * (c + g);
      if (i % a.N == 0 && a.s_out) a.s_out[b] = sab;
    }
  }
}

hipError_t launch_q_sample(const QArgs& a, hipStream_t s) {
  const int64_t total = a.B * a.N;
  if (total <= 0) return hipSuccess;
  const dim3 grid((unsigned)std::min<int64_t>((total + 255) / 256, 16384));
  hipLaunchKernelGGL(q_sample_kernel, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sddm
