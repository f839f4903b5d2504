// GaussianDiffusion schedule tables (model/diffusion.py:49-161) computed on the host with the
// rounding torch uses on CPU (SURVEY.md §8a "Numerical facts"):
//   torch.linspace(fp32): step in fp32, element i < n/2 = fmaf(step, i, start), else
//                         fmaf(-step, n-1-i, end);
//   torch.cumprod(fp32):  float64 running product rounded per element;
//   every other op:       one IEEE fp32 operation (no contraction), x**0.5 = sqrtf, x**2 = x*x.
// betas / alphas / alpha_bar are bit-exact with the reference; the sqrt-derived tables agree to
// the few-ulp inaccuracy of torch's own CPU sqrtf (tests/test_schedule.py).
#pragma clang fp contract(off)
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

namespace sddm {

static std::vector<float> linspace_f32(double start, double end, int n) {
  std::vector<float> out(n);
  const float s = (float)start, e = (float)end;
  if (n == 1) { out[0] = s; return out; }
  const float step = (e - s) / (float)(n - 1);
  const int half = n / 2;
  for (int i = 0; i < n; ++i)
    out[i] = i < half ? std::fma(step, (float)i, s) : std::fma(-step, (float)(n - 1 - i), e);
  return out;
}

// Returns 0 on success, 1 for an unknown schedule (NotImplementedError, diffusion.py:84).
int compute_schedule(const std::string& schedule, int T, double linear_start, double linear_end,
                     float* out /* [14][T+1] */) {
  const int L = T + 1;
  std::vector<float> betas(L, 0.f), alphas(L), ab(L);
  if (schedule == "linear" || schedule == "quad") {
    std::vector<float> lin = schedule == "linear"
                                 ? linspace_f32(linear_start, linear_end, T)
                                 : linspace_f32(std::sqrt(linear_start), std::sqrt(linear_end), T);
    for (int i = 0; i < T; ++i) betas[i + 1] = schedule == "linear" ? lin[i] : lin[i] * lin[i];
    for (int i = 0; i < L; ++i) alphas[i] = 1.0f - betas[i];
    double acc = 1.0;
    for (int i = 0; i < L; ++i) { acc *= (double)alphas[i]; ab[i] = (float)acc; }
  } else if (schedule == "cosine") {
    std::vector<float> f(L);
    const float s8 = 0.008f, den = (float)(1 + 0.008), hp = (float)(M_PI / 2);
    for (int i = 0; i < L; ++i) {
      const float ts = (float)i / (float)T + s8;
      const float x = ts / den * hp;
      const float c = (float)std::cos((double)x);
      f[i] = c * c;
    }
    for (int i = 0; i < L; ++i) ab[i] = f[i] / f[0];
    for (int i = 1; i < L; ++i) betas[i] = 1.0f - ab[i] / ab[i - 1];
    for (int i = 0; i < L; ++i) { if (betas[i] > 0.999f) betas[i] = 0.999f; alphas[i] = 1.0f - betas[i]; }
  } else {
    return 1;
  }
  std::vector<float> sab(L), sigma(L, 0.f), pnc(L, 0.f), sg(L, 0.f), ssh(L, 0.f), m(L), delta(L),
      sdelta(L), cxt(L, 0.f), cyt(L, 0.f), cep(L, 0.f), sde(L, 0.f);
  for (int i = 0; i < L; ++i) sab[i] = std::sqrt(ab[i]);
  for (int i = 1; i < L; ++i) {
    sigma[i] = std::sqrt((1.0f - ab[i - 1]) / (1.0f - ab[i]) * betas[i]);
    pnc[i] = betas[i] / std::sqrt(1.0f - ab[i]);
  }
  if (L > 1) sg[1] = 0.2f;
  for (int i = 2; i < L; ++i) sg[i] = sigma[i];
  for (int i = 1; i < L; ++i) ssh[i] = sigma[i] - sg[i] / std::sqrt(alphas[i]);
  for (int i = 0; i < L; ++i) {
    m[i] = std::sqrt((1.0f - ab[i]) / sab[i]);
    delta[i] = (1.0f - ab[i]) - (m[i] * m[i]) * ab[i];
    sdelta[i] = std::sqrt(delta[i]);
  }
  for (int i = 1; i < L; ++i) {
    const float omr = (1.0f - m[i]) / (1.0f - m[i - 1]);
    const float atd = alphas[i] * delta[i - 1];
    const float dtg = delta[i] - (omr * omr) * atd;
    const float sqa = std::sqrt(alphas[i]);
    cxt[i] = omr * delta[i - 1] / delta[i] * sqa + (1.0f - m[i - 1]) * (dtg / delta[i]) * (1.0f / sqa);
    cyt[i] = (m[i - 1] * delta[i] - m[i] * omr * atd) * sab[i - 1] / delta[i];
    cep[i] = (1.0f - m[i - 1]) * dtg / delta[i] * std::sqrt(1.0f - ab[i]) / sqa;
    sde[i] = std::sqrt(dtg * delta[i - 1] / delta[i]);
  }
  const std::vector<float>* tabs[14] = {&betas, &alphas, &ab, &sab, &pnc, &sigma, &sg, &ssh,
                                         &m, &sdelta, &cxt, &cyt, &cep, &sde};
  for (int k = 0; k < 14; ++k) std::memcpy(out + (size_t)k * L, tabs[k]->data(), sizeof(float) * L);
  return 0;
}

}  // namespace sddm
