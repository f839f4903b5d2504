// Kernel argument structs and host launchers (implemented in kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sddm {

// ---- noise-level embedding + every ResnetBlock's FeatureWiseAffine (UNetModified2.py:49-89) ----
struct EmbedArgs {
  const float* noise_levels;  // [R] explicit noise levels, or null -> use table / time step
  const float* table;         // sqrt_alpha_bar [R] (noise_condition 'sqrt_alpha_bar'), or null
  int time_step_mode;         // 1: noise level = (float)r ('time_step', model.py:112)
  int R;                      // rows
  int dim;                    // inner_channel (embedding width, 32)
  const float* emb_vec;       // [dim/2] PositionalEncoding.embedding_vector
  const float* w1; const float* b1;  // Linear(dim, 4dim)
  const float* w2; const float* b2;  // Linear(4dim, dim)
  const float* pw; const float* pb;  // concatenated FeatureWiseAffine Linears [SC][dim], [SC] (+conv1 bias)
  int SC;                     // sum of projected channels
  float* out;                 // [R][SC]
};
hipError_t launch_embed(const EmbedArgs& a, hipStream_t s);

// ---- GroupNorm statistics finalize (nn.GroupNorm, UNetModified2.py:117) ----
struct GNSrc { const float* stats; int C; int tiles; int n_tile; };
struct GNArgs {
  GNSrc a, b;                 // virtual concat of two producers (b.C == 0 if none)
  const float* gamma; const float* beta;
  int G; float eps; int B;
  float* scale; float* shift; // [B][Ca+Cb]
};
hipError_t launch_gn_finalize(const GNArgs& a, hipStream_t s);

// ---- framing + first Conv2d(2 -> C) (UNetModified2.py:23-28, 177-178, 244-247) ----
struct ConvInArgs {
  const float* cond; const float* x;  // [B][N] fp32
  int N, F, W, S;             // samples, frames, segment_len, segment_stride
  int Cout;                   // 32
  const float* w;             // [Cout][2][3][3] fp32
  const float* bias;          // [Cout]
  void* out;                  // [B][F][W][Cout] (T)
  float* stats;               // [B][tiles][Cout][2]
  int TR;                     // frame rows per block
  int* t_dev;                 // step counter decremented once per launch (may be null)
  unsigned long long* stamps; // SDDM_STAMPS builds only
};
hipError_t launch_conv_in(int dtype, const ConvInArgs& a, int B, hipStream_t s);

// ---- MFMA implicit-GEMM 3x3 convolution (Block / Downsample / Upsample / ResnetBlock) ----
struct GNFuse;
struct ConvArgs {
  const void* srcA; const void* srcB; int CA, CB;  // virtual channel concat (UNetModified2.py:263)
  int Hi, Wi;                 // stored source dims
  int Ho, Wo;                 // output dims
  int upsample;               // stride-1 kernel reads a nearest-2x upsampled source (UNetModified2.py:96-100)
  int TR, TW, tiles_x, n_tiles;
  // GroupNorm + SiLU prologue (Block, UNetModified2.py:116-120): the producer's per-tile statistics
  // are finalized in the consumer (gamma == null: no GN / SiLU)
  const float* gstA; int gtilesA, gntileA;
  const float* gstB; int gtilesB, gntileB;
  const float* gamma; const float* beta; int groups; float eps;
  const void* wgt;            // packed [Cout_pad][Cin/32][9][32] (T)
  const float* bias;          // [Cout]
  const float* temb; int temb_ld; const int* t_dev; int temb_per_b;  // + temb row (ResnetBlock.noise_func)
  int Cout;
  int res_mode;               // 0 none, 1 identity (res_src [B][Ho][Wo][Cout]), 2 conv1x1 over raw concat
  const void* res_src;        // identity residual
  const void* rawA; const void* rawB; int RCA, RCB;  // 1x1 residual input (ResnetBlock.res_conv, UNetModified2.py:135)
  const void* res_wgt;        // packed [Cout_pad][RCA+RCB] (T)
  void* out;                  // [B][Ho][Wo][Cout]
  float* stats;               // [B][n_tiles][Cout][2] (sum, M2 about tile mean) or null
  int deep_zin;               // conv_deep: 1 = a tile's channel blocks on one XCD (input halo from L2), 0 = z-major
  int deep_nw;                // conv_deep: waves per block (4: two blocks per CU, 8: one)
  int deep_nb;                // conv_deep: output channels per block (32 or 16; 0 = 32)
  unsigned long long* stamps; // SDDM_STAMPS builds only: per-block phase timestamps [blocks][8]
  int dbg;                    // ablation flags for timing experiments (0 in production); conv_deep: 1 no GN
                              // finalize, 2 no GN+SiLU, 4 no staging loads, 8 no K loop, 16 no stats, 32 no weight loads
  // conv_tile (16-bit dtypes): chunk-major weight images, one 16-byte unit = 8 input channels of
  // one output channel: 3x3 [Cin/32][9][4][Cout][8], res_conv [RC/32][4][Cout][8]
  const void* wgt_t;
  const void* res_wgt_t;
  // conv_deep: MFMA-fragment-major weight images, one 64-lane A fragment contiguous:
  // 3x3 [Cout/16][Cin/32 * 9][64 lanes][8], res_conv [Cout/16][RC/32][64 lanes][8]
  const void* wgt_f;
  const void* res_wgt_f;
};

// ---- the UNet's bottom level in one launch (conv_chain.hip, bf16 / f16): downs.<last> (stride-2),
// mid.0 (ResnetBlock, identity residual), ups.0 (ResnetBlock over cat(mid, downs.<last>), res_conv)
struct ChainArgs {
  const void* x;              // [B][2H][2W][C] the level's input (downs.<last-1> output)
  void* out;                  // [B][H][W][C] ups.0.block2 output
  const void* wgt[5];         // MFMA-fragment-major 3x3 images (ConvArgs::wgt_f layout) of the five convs
  const void* res_wgt;        // ups.0 res_conv, [C/16][2C/32][64 lanes][8]
  const float* bias[5];       // (ups.0.block2's includes the res_conv bias)
  const float* gamma[4]; const float* beta[4];   // GroupNorm of mid.0.block1/2, ups.0.block1 (2C), ups.0.block2
  const float* temb[2];       // noise-embedding projection of mid.0 / ups.0 (row stride temb_ld)
  int temb_ld; const int* t_dev; int temb_per_b;
  int C, H, W, groups; float eps;
};
hipError_t launch_conv_chain(int dtype, const ChainArgs& a, int B, hipStream_t s);

// ---- K-streamed implicit-GEMM tile convolution (conv_tile.hip, bf16 / f16 only) ----
// cfg: tile configuration index (kTileCfgs in conv_tile.hip); s2: stride-2 Downsample
struct TileCfg { int wpx, wco, fp, fc; };   // waves along pixels / channels, 16-wide fragments per wave
int conv_tile_ncfg();
TileCfg conv_tile_cfg(int cfg);
hipError_t launch_conv_tile(int dtype, int cfg, bool s2, const ConvArgs& a, int B, hipStream_t s);
size_t conv_tile_lds_bytes(int cfg, bool s2, const ConvArgs& a);

// ---- whole-K-resident tile convolution for the narrow levels (conv_deep.hip) ----
// mt: output pixels per block (32 / 64 / 128); s2: stride-2 Downsample
hipError_t launch_conv_deep(int dtype, int mt, bool s2, const ConvArgs& a, int B, hipStream_t s);
size_t conv_deep_lds_bytes(int dtype, int mt, bool s2, const ConvArgs& a);
int conv_deep_ring_depth(int dtype, int mt, int nw, int ksteps, int nb);   // the D template argument (profiles)

// LDS per workgroup every launcher and planner sizes against: gfx950's 160 KiB (sddm_create fails
// on a device that offers less, so no plan is built for LDS the device does not have)
constexpr int kLdsBytes = 160 * 1024;

// ---- row-streaming 3x3 convolution for segment widths 64 / 128 (conv_strip.hip) ----
hipError_t launch_conv_strip(int dtype, int nblk, int mpi, int SR, const ConvArgs& a, int B, hipStream_t s);
size_t conv_strip_lds_bytes(int dtype, int nblk, int mpi, const ConvArgs& a);

// ---- final Block(C -> 1) + overlapAdd + p_transition (UNetModified2.py:235,267-268; diffusion.py:164-223) ----
struct TransCoef {            // device pointers to the GaussianDiffusion buffers [T+1]
  const float* betas; const float* alphas; const float* sqrt_alpha_bar; const float* pnc;
  const float* sigma; const float* sgamma; const float* ssh; const float* sqrt_delta;
  const float* c_xt; const float* c_yt; const float* c_epst; const float* sde;
};
struct StepParams { int t; int pad; uint64_t seed; int64_t row_offset; };   // device-side, per sample call
hipError_t launch_set_params(StepParams* p, int t, uint64_t seed, int64_t row_offset, hipStream_t s);

struct FinalArgs {
  const void* src; int C;     // [B][F][W][C] (T)
  const float* gst; int gtiles, gntile;          // producer tile statistics (final_conv GroupNorm)
  const float* gamma; const float* beta; int groups; float eps;
  const float* w; float bias; // [C][3][3] fp32 (out_channel = 1)
  int N, F, W, S, FT;
  int mode;                   // -1: write eps (network forward); else sddm_transition mode
  float* eps_out;             // mode -1
  float* x;                   // [B][N] state, updated in place
  const float* cond;          // [B][N]
  const int* t_dev;
  TransCoef co;
  uint64_t seed; int64_t row_offset;
  const StepParams* sp;       // when set, seed / row_offset come from device memory (graph replay)
  const float* noise; int64_t noise_ld;   // caller-supplied draws (TransArgs), row b of draw t at noise[t * noise_ld + b * N]
  unsigned long long* stamps; // SDDM_STAMPS builds only
};
hipError_t launch_final(int dtype, const FinalArgs& a, int B, hipStream_t s);

// ---- standalone transition / initial state (diffusion.py:164-223, 281-320; model.py:57-68) ----
// noise (nullable): caller-supplied standard-normal draws [draw][noise_ld] (sddm_sample_noise): draw 0 is
// x_T's, draw t the transition's at step t, element i of a draw at noise[draw * noise_ld + i] (i = the
// call-local flat index); null = the Philox stream keyed by (seed, draw, global element)
struct TransArgs {
  int mode; const float* x_t; const float* eps; const float* cond; float* out;
  int64_t total; int64_t N; int t; const int* t_dev; TransCoef co; uint64_t seed; int64_t row_offset;
  const float* noise; int64_t noise_ld;
};
hipError_t launch_transition(const TransArgs& a, hipStream_t s);
struct InitArgs {
  int mode; const float* cond; float* out; int64_t total; int64_t N; int T; TransCoef co; uint64_t seed; int64_t row_offset;
  const float* noise;         // caller-supplied draw 0 (nullable), element i at noise[i]
};
hipError_t launch_init_state(const InitArgs& a, hipStream_t s);
hipError_t launch_set_int(int* p, int v, hipStream_t s);
hipError_t launch_delay(unsigned us, hipStream_t s);   // bounded busy wait (lane phase offsets)

// ---- DiffWave (reference model/diffwave.py; diffwave.hip) ----
struct DWEmbedArgs {          // DiffusionEmbedding + every layer's diffusion_projection, rows r = 0..R-1
  const float* noise_levels;  // [R] explicit, or null -> time_step (r) / table[r]
  const float* table; int time_step_mode; int R;
  const float* emb_vec;       // [64]
  const float* w1; const float* b1; const float* w2; const float* b2;   // 128->512, 512->512
  const float* pw; const float* pb; int L;                               // [L*64][512], [L*64]
  float* out;                 // [R][L][64]
};
hipError_t launch_dw_embed(const DWEmbedArgs& a, hipStream_t s);
struct DWUpArgs {             // SpectrogramUpsampler: spec [B][H][F] -> out [B][256F][Kp] (T)
  const float* spec; float* mid; void* out; int B, H, F, Kp;
  const float* k1; const float* b1; const float* k2; const float* b2;
};
hipError_t launch_dw_upsample(int dtype, const DWUpArgs& a, hipStream_t s);
struct DWCondArgs {           // cond[l][b][n][128] = Wc[l] spec[b][n] + bc[l]
  const void* spec; const void* w; const float* bias; void* out; int B, N, L, Kp;
};
hipError_t launch_dw_cond(int dtype, const DWCondArgs& a, hipStream_t s);
struct DWInArgs { const float* audio; const float* w; const float* b; void* x; int64_t total; int* t_dev; };
hipError_t launch_dw_input(int dtype, const DWInArgs& a, hipStream_t s);
struct DWLayerArgs {
  const void* x_in; void* x_out; void* z; int first;   // z: gated activations [L][B][N][64] (T)
  const void* cond; int layer, L;
  const float* ds; const int* t_dev; int ds_per_b;   // [rows][L][64]
  const void* w1; const float* b1;                   // dilated conv [128][3*64] (k = tap*64 + ci), bias [128]
  const void* w2; const float* b2;                   // output_residual [64][64] (rows 0-63 used), bias
  int dil, N, B;
};
hipError_t launch_dw_layer(int dtype, const DWLayerArgs& a, hipStream_t s);
size_t dw_layer_lds_bytes(int dtype);
struct DWSkipArgs {           // skip[b][n][64] = Wo_all [64][L*64] z[b][n][L*64] + bias_sum (fp32 out)
  const void* z; const void* w; const float* bias; float* skip; int B, N, L;
};
hipError_t launch_dw_skip(int dtype, const DWSkipArgs& a, hipStream_t s);
struct DWOutArgs {
  const float* skip; const float* wsp; const float* bsp; const float* wop; const float* bop;
  float sqrt_layers; float* eps; int64_t total;
};
hipError_t launch_dw_output(const DWOutArgs& a, hipStream_t s);

}  // namespace sddm
