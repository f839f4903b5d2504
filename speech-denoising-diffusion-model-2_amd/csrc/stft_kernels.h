// Log-magnitude spectrogram featurizer (reference prepare_spectrogram.py:20-55, through
// torchaudio.transforms.Spectrogram / MelSpectrogram).
#pragma once
#include "sddm_common.h"

namespace sddm {

// out[b][m][f] = clamp((log10(S[b][m][f]) - 1 + 5) / 5, 0, 1) with
//   S = |rfft(window * frame_f)| / sqrt(sum window^2)            (power 1, normalized, n_fft taps)
//   frame_f = audio[b][f * hop - n_fft/2 + n], reflect-padded       (center=True, pad_mode reflect)
//   and, when fb != null, S_mel[m] = sum_k fb[k][m] S[k]           (MelScale, fb [n_fft/2+1][n_out])
struct StftArgs {
  const float* audio; int64_t B, N; int n_fft, hop, frames, n_out;
  const float* window; const float* fb; float* out;
};
hipError_t launch_stft_features(const StftArgs& a, hipStream_t s);

}  // namespace sddm
