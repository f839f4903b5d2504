/* sddm_hip.h — C ABI of libsddm_hip.so, the MI355X-native reverse-diffusion sampler.
 *
 * The reference exposes this path only as a Python plugin API: objects are
 * built by ConfigParser.init_obj (parse_config.py:82-95) from the "arch" / "diffusion" /
 * "network" blocks of config.json, weights arrive through load_state_dict (infer.py:46-51) and
 * the hot loop is entered through model.infer(condition) (infer.py:77, trainer/trainer.py:115).
 * Each entry point below replaces one piece of that surface; the Python facade in
 * speech-denoising-diffusion-model-2_amd/model/ binds them with ctypes.
 *
 * Conventions
 *  - every function returns 0 (SDDM_OK) or a status code; sddm_last_error() gives the
 *    thread-local message.  The facade maps SDDM_ERR_NOT_IMPLEMENTED to NotImplementedError,
 *    SDDM_ERR_SHAPE / SDDM_ERR_INVALID_ARG to AssertionError / ValueError like the reference
 *    (diffusion.py:84, model.py:17-26, UNetModified2.py:13), others to RuntimeError.
 *  - device pointers (cond, x_t, out, spec) are owned by the caller; the library owns weights,
 *    schedule tables and workspace.  `stream` is a hipStream_t (NULL = default stream); calls
 *    are asynchronous with respect to the host and ordered on that stream.
 *  - one context per device; a context must not be used from two threads at once.
 */
#ifndef SDDM_HIP_H
#define SDDM_HIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDDM_ABI_VERSION 1

enum sddm_status {
  SDDM_OK = 0,
  SDDM_ERR_NOT_IMPLEMENTED = 1, /* unknown schedule / transition / network type          */
  SDDM_ERR_INVALID_ARG = 2,     /* bad argument value, unknown parameter key             */
  SDDM_ERR_SHAPE = 3,           /* geometry the network cannot take (UNetModified2.py:13) */
  SDDM_ERR_HIP = 4,             /* HIP runtime error                                     */
  SDDM_ERR_STATE = 5            /* called before configure / missing parameters          */
};

enum sddm_dtype { SDDM_F32 = 0, SDDM_BF16 = 1, SDDM_F16 = 2 };

/* p_transition modes of SDDM (model/model.py:20-23, diffusion.py:164-223) */
enum sddm_transition {
  SDDM_TR_ORIGINAL = 0,     /* 'original' and 'condition_in' share p_transition */
  SDDM_TR_SR3 = 1,
  SDDM_TR_SUPPORTIVE = 2,
  SDDM_TR_CONDITIONAL = 3
};

typedef struct sddm_ctx sddm_ctx;

int sddm_abi_version(void);
const char* sddm_last_error(void);

/* Replaces `device = torch.device(...)` + the dtype choice (infer.py:36).
 * compute_dtype: storage/MFMA dtype of network activations (sddm_dtype); state stays fp32. */
int sddm_create(int device, int compute_dtype, sddm_ctx** out);
void sddm_destroy(sddm_ctx* ctx);

/* Replaces config.init_obj('diffusion'|'network'|'arch', ...) (infer.py:37-39,
 * parse_config.py:82-95).  `json` is {"arch": {...}, "diffusion": {...}, "network": {...},
 * "num_samples": N} with the reference's type names and args verbatim
 * (config_unet.json, config_diffwave.json, config_wavegrad.json). */
int sddm_configure(sddm_ctx* ctx, const char* json);

/* Replaces model.load_state_dict(state_dict) (infer.py:51) one tensor at a time.  `key` is
 * the reference state_dict key ("noise_estimate_model.downs.1.block1.block.3.weight",
 * "diffusion.sigma", with or without a DataParallel "module." prefix).  host_ptr holds a
 * contiguous tensor of `src_dtype` (sddm_dtype) with the reference shape. */
int sddm_load_param(sddm_ctx* ctx, const char* key, const void* host_ptr, const int64_t* shape,
                    int ndim, int src_dtype);

/* Number of parameters still missing (0 when the network is complete). */
int sddm_missing_params(sddm_ctx* ctx, int64_t* n_missing);

/* Replaces SDDM.infer(condition) (model/model.py:50-124; SDDM_spectrogram.infer model.py:212-257
 * when the arch is SDDM_spectrogram, then `cond` is the spectrogram [B, bins, frames]).
 * cond: [B, 1, N] fp32 device; out: [B, 1, N] fp32 device (x_0).  Noise is the counter-based
 * stream keyed by (seed, draw, (row_offset + b) * N + n) so a row block sampled on any rank
 * equals the same rows of a single-device run. */
int sddm_sample(sddm_ctx* ctx, const float* cond, int64_t B, int64_t N, uint64_t seed,
                int64_t row_offset, float* out, void* stream);

/* SURVEY.md §8(b) noise_mode 1: as sddm_sample, but every Gaussian draw comes from the caller, so the
 * loop reproduces the reference's own torch.randn_like draws bit for bit (model.py:57-68,
 * diffusion.py:172,187,207,220,285,306).  noise: [T + 1][B][N] fp32 device; draw 0 is x_T's noise
 * (unused by 'supportive' and by modes starting from the condition), draw t the transition noise of
 * step t (read for t >= 2 only).  The draws are consumed in the reference's order (x_T, then
 * t = T .. 2), so model.model.reference_noise() stacks torch.randn_like calls into this layout. */
int sddm_sample_noise(sddm_ctx* ctx, const float* cond, int64_t B, int64_t N, const float* noise, float* out,
                      void* stream);

/* SDDM.infer(condition, continuous=True) (model/model.py:79-103): as sddm_sample, and after the
 * step at t, whenever t % sample_inter == 0, x_{t-1} is copied to the next slot of `record`
 * ([T / sample_inter][B][N] fp32 device).  sample_inter = 1 | (T // 100) (model.py:72). */
int sddm_sample_continuous(sddm_ctx* ctx, const float* cond, int64_t B, int64_t N, uint64_t seed,
                           int64_t row_offset, float* out, float* record, int sample_inter, void* stream);

/* Replaces one noise_estimate_model(condition, x_t, noise_level) call (model.py:110):
 * noise_level: [B] fp32 device.  eps_out: [B, 1, N] fp32 device. */
int sddm_network_forward(sddm_ctx* ctx, const float* cond, const float* x_t,
                         const float* noise_level, int64_t B, int64_t N, float* eps_out,
                         void* stream);

/* Replaces diffusion.p_transition*(x_t, t, predicted[, condition]) (diffusion.py:164-223).
 * cond may be NULL for modes that do not read it. */
int sddm_transition(sddm_ctx* ctx, int mode, const float* x_t, const float* eps,
                    const float* cond, int t, int64_t B, int64_t N, uint64_t seed,
                    int64_t row_offset, float* out, void* stream);

/* Replaces diffusion.q_stochastic (mode 0, diffusion.py:225-251) and
 * q_stochastic_conditional (mode 1, diffusion.py:253-279), the forward-process noising of the
 * training step.  x0 / y / noise / x_t / combined: [B][N] fp32 device pointers; t: [B] int64
 * device (drawn by the caller, torch.randint(1, T+1) in the reference); r: [B] fp32 device
 * uniform draws (mode 0; NULL = t_is_integer).  Outputs: x_t; combined noise (mode 1, nullable);
 * s_out[B] = the sqrt_alpha_bar sample; level_out[B] = t + r (mode 0, nullable). */
int sddm_q_sample(sddm_ctx* ctx, int mode, const float* x0, const float* y, const float* noise,
                  const int64_t* t, const float* r, int64_t B, int64_t N, float* x_t,
                  float* combined, float* s_out, float* level_out, void* stream);

/* Measured per-layer conv kernels (no reference counterpart: a tuning table).  json = one table
 * {"lane_batch": B, "dtype": "bfloat16", "num_samples": N, "kernel": {"<layer name>": "strip" |
 * "tile:<cfg>" | "deep:<pixels>:<waves>:<channels>", ...}} or {"tables": [table, ...]}; at the next
 * plan build the first table whose lane batch / dtype / num_samples match the plan applies; a
 * float16 plan with no float16 table takes a matching bfloat16 one (never the reverse); none
 * otherwise (and per layer whenever the requested kernel does not fit that layer). */
int sddm_set_conv_tuning(sddm_ctx* ctx, const char* json);

/* Replaces the torchaudio featurizer of prepare_spectrogram.py:20-55 (context-free):
 * out[B][n_out][1 + N/hop] = clamp((log10(S) - 1 + 5) / 5, 0, 1), S = |STFT| (center, reflect
 * padding, `window` [n_fft], power 1, normalized by sqrt(sum window^2)); with fb
 * ([n_fft/2+1][n_out], nullable) S is projected onto the mel filterbank first.  All pointers are
 * device pointers; n_fft a power of two <= 1024. */
int sddm_log_spectrogram(const float* audio, int64_t B, int64_t N, int n_fft, int hop,
                         const float* window, const float* fb, int n_out, float* out, void* stream);

/* Replaces diffusion.get_x_T / get_x_T_conditional / randn_like (model.py:57-68). */
int sddm_initial_state(sddm_ctx* ctx, int mode, const float* cond, int64_t B, int64_t N,
                       uint64_t seed, int64_t row_offset, float* out, void* stream);

/* Host-only: the 14 GaussianDiffusion buffers (diffusion.py:50-161) for a schedule, written
 * as out[14][n_timestep+1] in registration order (betas, alphas, alpha_bar, sqrt_alpha_bar,
 * predicted_noise_coeff, sigma, supportive_gamma, supportive_sigma_hat, m, sqrt_delta, c_xt,
 * c_yt, c_epst, sqrt_delta_estimated). */
int sddm_schedule(const char* schedule, int n_timestep, double linear_start, double linear_end,
                  float* out);

/* Timing of the last sddm_sample's dominant kernel class (HIP events on the sampling stream):
 * average duration in ms of the UNet 3x3 convolution launches, and how many were timed. */
int sddm_profile_enable(sddm_ctx* ctx, int enable);
int sddm_profile_read(sddm_ctx* ctx, const char* kernel_class, double* avg_ms, int64_t* launches,
                      double* bytes_per_launch, double* flops_per_launch);
/* Per-op breakdown of the timed launches as a JSON array written into buf. */
int sddm_profile_ops(sddm_ctx* ctx, char* buf, int64_t buflen);

#ifdef __cplusplus
}
#endif
#endif /* SDDM_HIP_H */
