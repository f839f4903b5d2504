// WaveGrad kernel argument structs and host launchers (implemented in wavegrad.hip).
#pragma once
#include "sddm_common.h"

namespace sddm {

// One WaveGrad convolution (reference model/wavegrad.py) as an implicit GEMM over (tap, ci):
//   out[b][t][co] = post( bias[co] + sum_{tap, ci} W[co][tap][ci] * pre(src[b][map(t')][ci]) ) (+ res)
//   t' = t + (tap - (K-1)/2) * dil, zero outside [0, Tc) (the conv's zero padding, applied after
//   F.interpolate); map = identity | nearest up (t' / f) | nearest down (t' * f).
// pre:  0 none | 1 leaky_relu(0.2) | 2 leaky_relu(0.2)(shift + scale * x), shift / scale from a FiLM
//       output [B][Tc][2 Cin] (shift = channels [0, Cin), scale = [Cin, 2 Cin)).
// post: 0 none | 1 leaky_relu(0.2) then + enc[row][co] (FiLM input_conv + PositionalEncoding).
// res:  + res[b][rmap(t)][co] (DBlock residual_dense, UBlock block1 / x), rmap identity or up.
enum { WG_MAP_ID = 0, WG_MAP_UP = 1, WG_MAP_DOWN = 2 };
// positions per WaveGrad conv launch: the staging index map (wg_map) is exact below 2^23
constexpr int kWgMaxPositions = 1 << 23;
struct WGConvArgs {
  const void* src; int src_T, src_C, map, f;   // source [B][src_T][src_C] (T); channels [0, Cin) are read
  int Tc, Cin, K, dil, pre;
  const void* film;                            // [B][Tc][2 Cin] (T) for pre == 2
  const void* w; const float* bias; int Cout;  // packed [Cout_pad64][K][Cin] (T), bias [Cout] fp32
  int post; const float* enc; int enc_stride, enc_off, enc_per_b; const int* t_dev;   // enc [rows][stride]
  const void* res; int res_map, res_f, res_T;  // [B][res_T][Cout] (T) or null
  void* out; int out_f32;                      // [B][Tc][Cout] (T, or fp32 when out_f32)
  int B;
  // FiLM of the NEXT conv's input applied in this conv's epilogue (16-bit / fp32 storage, Cout % 4
  // == 0): m = leaky(shift + scale * v) with efilm [B][Tc][2 Cout] (shift | scale).  post_film 1:
  // out <- m (v is consumed only through the FiLM); 2: out <- v and out2 <- m (v is also a residual)
  const void* efilm; void* out2; int post_film;
};
hipError_t launch_wg_conv(int dtype, const WGConvArgs& a, hipStream_t s);
// true when launch_wg_conv takes the LDS-staged kernel (which applies pre == 2 itself)
bool wg_conv_uses_lds(const WGConvArgs& a);

// downsample.0: Conv1d(1, 32, 5, padding=2) on the fp32 audio [B][N] -> [B][N][32] (T); decrements
// the device step counter (one launch per reverse step)
struct WGFirstArgs { const float* audio; const float* w; const float* b; void* out; int B, N; int* t_dev; };
hipError_t launch_wg_first(int dtype, const WGFirstArgs& a, hipStream_t s);

// FiLM modulation materialised once per element: u[b][t][c] = leaky_relu(0.2)(shift + scale * x)
// (wavegrad.py:98-99, 104-105, 107-108); film [B][T][2C] (shift | scale), x / u [B][T][C]
struct WGFilmArgs { const void* x; const void* film; void* out; int64_t BT; int C; };
hipError_t launch_wg_film(int dtype, const WGFilmArgs& a, hipStream_t s);

// spectrogram [B][C][F] fp32 -> [B][F][C] (T)
struct WGSpecArgs { const float* spec; void* out; int B, C, F; };
hipError_t launch_wg_spec(int dtype, const WGSpecArgs& a, hipStream_t s);

// PositionalEncoding rows of the 5 FiLMs: enc[r][off_i + k] = sin / cos(nl_r * ev_i[k]) (wavegrad.py:44-49)
struct WGEncArgs {
  const float* noise_levels;   // [R] explicit, or null -> table[r] (sqrt_alpha_bar) / r (time_step)
  const float* table; int time_step_mode; int R;
  const float* ev; int stride; int n; int dims[5]; int offs[5];   // ev: concatenated exp vectors
  float* out;
};
hipError_t launch_wg_enc(const WGEncArgs& a, hipStream_t s);

}  // namespace sddm
