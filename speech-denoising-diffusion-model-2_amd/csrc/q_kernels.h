// Forward-process (training-side) noising kernels, reference model/diffusion.py:225-279.
#pragma once
#include "sddm_common.h"

namespace sddm {

// mode 0, q_stochastic (diffusion.py:225-251), per row b with t_b = t[b], r_b = r[b]:
//   s = sab[t-1] + r (sab[t] - sab[t-1])   (r = null: t_is_integer, s = sab[t])
//   x_t = s x_0 + sqrt(1 - s^2) noise;  s_out[b] = s, level_out[b] = t + r
// mode 1, q_stochastic_conditional (diffusion.py:253-279):
//   g = sqrt_delta[t] noise, c = m[t] sab[t] (y - x_0)
//   x_t = sab[t] x_0 + c + g;  combined = 1 / sqrt(1 - alpha_bar[t]) (c + g);  s_out[b] = sab[t]
struct QArgs {
  int mode;
  const float* x0; const float* y; const float* noise; const int64_t* t; const float* r;
  const float* sab; const float* alpha_bar; const float* m; const float* sqrt_delta;
  float* x_t; float* combined; float* s_out; float* level_out;
  int64_t B, N;
};
hipError_t launch_q_sample(const QArgs& a, hipStream_t s);

}  // namespace sddm
