// Log-magnitude (mel) spectrogram featurizer, reference prepare_spectrogram.py:20-55.
// One block per (frame, clip): the windowed, reflect-padded frame and the twiddle table sit in
// LDS, every thread evaluates DFT bins k = tid, tid + 256, ... as exact-index sums
// (twiddle[(n k) mod n_fft], fp32 accumulation), the magnitudes go back to LDS for the mel
// projection, and the log / clamp epilogue writes [B][n_out][frames].
#include "stft_kernels.h"

namespace sddm {

constexpr int STFT_MAX_FFT = 1024;

__global__ __launch_bounds__(256) void stft_kernel(StftArgs a) {
#pragma clang fp contract(off)
  __shared__ float xs[STFT_MAX_FFT], cs[STFT_MAX_FFT], sn[STFT_MAX_FFT], mag[STFT_MAX_FFT / 2 + 1];
  const int f = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, nf = a.n_fft, nb = nf / 2 + 1;
  const float* x = a.audio + (size_t)b * a.N;
  float wsum = 0.f;
  for (int n = tid; n < nf; n += 256) {
    int64_t i = (int64_t)f * a.hop - nf / 2 + n;               // center=True, reflect padding
    if (i < 0) i = -i;
    if (i >= a.N) i = 2 * (a.N - 1) - i;
    xs[n] = a.window[n] * x[i];
    float s, c;
    sincospif(2.0f * (float)n / (float)nf, &s, &c);
    cs[n] = c;
    sn[n] = s;
  }
  for (int n = 0; n < nf; ++n) wsum += a.window[n] * a.window[n];   // uniform; tiny
  const float norm = sqrtf(wsum);
  __syncthreads();
  for (int k = tid; k < nb; k += 256) {
    float re = 0.f, im = 0.f;
    for (int n = 0; n < nf; ++n) {
      const int j = (n * k) & (nf - 1);
      re += xs[n] * cs[j];
      im -= xs[n] * sn[j];
    }
    mag[k] = sqrtf(re * re + im * im) / norm;
  }
  __syncthreads();
  for (int m = tid; m < a.n_out; m += 256) {
    float v;
    if (a.fb) {
      v = 0.f;
      for (int k = 0; k < nb; ++k) v += mag[k] * a.fb[(size_t)k * a.n_out + m];
    } else {
      v = mag[m];
    }
    float l = log10f(v) - 1.f;
    l = (l + 5.f) / 5.f;
    l = fminf(fmaxf(l, 0.f), 1.f);
    a.out[((size_t)b * a.n_out + m) * a.frames + f] = l;
  }
}

hipError_t launch_stft_features(const StftArgs& a, hipStream_t s) {
  if (a.n_fft < 2 || a.n_fft > STFT_MAX_FFT || (a.n_fft & (a.n_fft - 1)) || a.hop < 1 || a.N <= a.n_fft / 2 ||
      a.frames < 1 || a.B < 1)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(stft_kernel, dim3(a.frames, (unsigned)a.B), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace sddm
