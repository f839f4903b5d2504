// libsddm_hip runtime: context, parameter registry, weight packing, per-batch execution plan of
// one UNetModified2 reverse-diffusion step, and the C ABI declared in include/sddm_hip.h.
//
// Reference counterparts:
//   sddm_configure      ConfigParser.init_obj('diffusion'|'network'|'arch') (parse_config.py:82-95)
//   sddm_load_param     model.load_state_dict (infer.py:46-51)
//   sddm_sample         SDDM.infer (model/model.py:50-124)
//   sddm_network_forward UNetModified2.forward (model/UNetModified2.py:237-269)
//   sddm_transition     GaussianDiffusion.p_transition* (model/diffusion.py:164-223)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <memory>
#include <string>
#include <vector>

#include "../../include/sddm_hip.h"
#include "json_mini.h"
#include "kernels.h"
#include "q_kernels.h"
#include "stft_kernels.h"
#include "sddm_common.h"

namespace sddm {
int compute_schedule(const std::string& schedule, int T, double linear_start, double linear_end,
                     float* out);
}
using namespace sddm;

static thread_local std::string g_last_error;
static void sddm_set_error(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  (void)code;
}
#define FAIL(code, ...)                 \
  do {                                  \
    sddm_set_error(code, __VA_ARGS__);  \
    return code;                        \
  } while (0)

static const char* kTableNames[14] = {"betas", "alphas", "alpha_bar", "sqrt_alpha_bar",
                                      "predicted_noise_coeff", "sigma", "supportive_gamma",
                                      "supportive_sigma_hat", "m", "sqrt_delta", "c_xt", "c_yt",
                                      "c_epst", "sqrt_delta_estimated"};

// ---------------------------------------------------------------------------------------------
// fp32 -> storage dtype (round to nearest even) on the host
// ---------------------------------------------------------------------------------------------
static uint16_t f32_to_bf16_bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static uint16_t f32_to_f16_bits(float f) {
  _Float16 h = (_Float16)f;
  uint16_t r;
  std::memcpy(&r, &h, 2);
  return r;
}
static size_t dtype_size(int dt) { return dt == DT_F32 ? 4 : 2; }
static const char* dt_name(int dt) { return dt == DT_F32 ? "f32" : dt == DT_BF16 ? "bf16" : "f16"; }
static void store_elem(void* base, size_t idx, float v, int dt) {
  if (dt == DT_F32) ((float*)base)[idx] = v;
  else if (dt == DT_BF16) ((uint16_t*)base)[idx] = f32_to_bf16_bits(v);
  else ((uint16_t*)base)[idx] = f32_to_f16_bits(v);
}

// ---------------------------------------------------------------------------------------------
// device arena (one hipMalloc, bump allocation, 256-B alignment)
// ---------------------------------------------------------------------------------------------
struct Arena {
  char* base = nullptr;
  size_t cap = 0, used = 0;
  std::vector<std::pair<size_t, size_t>> pending;  // (offset, bytes) reservations before alloc
  size_t reserve(size_t bytes) {
    const size_t off = (used + 255) & ~(size_t)255;
    used = off + bytes;
    return off;
  }
  hipError_t commit() {
    if (base) { (void)hipFree(base); base = nullptr; }
    cap = used;
    if (cap == 0) return hipSuccess;
    hipError_t e = hipMalloc(&base, cap);
    if (e == hipSuccess) e = hipMemset(base, 0, cap);
    return e;
  }
  void reset() {
    if (base) (void)hipFree(base);
    base = nullptr; cap = used = 0;
  }
  template <typename T> T* at(size_t off) const { return (T*)(base + off); }
};

// ---------------------------------------------------------------------------------------------
// UNetModified2 architecture (UNetModified2.py:146-235)
// ---------------------------------------------------------------------------------------------
struct UNetCfg {
  int in_channel = 2, out_channel = 1, inner = 32, groups = 32, res_blocks = 3;
  std::vector<int> mults{1, 2, 3, 4, 5};
  int seg = 128, stride = 64;
  double dropout = 0.0;
};
struct LayerDesc { int kind; std::string name; int cin, cout; };  // kind 0 conv,1 res,2 down,3 up,4 final
static std::vector<LayerDesc> unet_layers(const UNetCfg& c, std::vector<LayerDesc>* downs_out,
                                          std::vector<LayerDesc>* mid_out, std::vector<LayerDesc>* ups_out) {
  std::vector<LayerDesc> downs, mid, ups;
  downs.push_back({0, "downs.0", c.in_channel, c.inner});
  std::vector<int> feat{c.inner};
  int cin = c.inner, idx = 1, cout = c.inner;
  for (size_t ind = 0; ind < c.mults.size(); ++ind) {
    cout = c.inner * c.mults[ind];
    for (int r = 0; r < c.res_blocks; ++r) {
      downs.push_back({1, "downs." + std::to_string(idx++), cin, cout});
      feat.push_back(cout);
      cin = cout;
    }
    downs.push_back({2, "downs." + std::to_string(idx++), cout, cout});
    feat.push_back(cout);
  }
  mid.push_back({1, "mid.0", cin, cin});
  idx = 0;
  for (int ind = (int)c.mults.size() - 1; ind >= 0; --ind) {
    cin = c.inner * c.mults[ind];
    cout = cin;
    ups.push_back({1, "ups." + std::to_string(idx++), cin + feat.back(), cout});
    feat.pop_back();
    ups.push_back({3, "ups." + std::to_string(idx++), cout, cout});
    cout = ind == 0 ? c.inner : c.inner * c.mults[ind - 1];
    for (int r = 0; r < c.res_blocks; ++r) {
      ups.push_back({1, "ups." + std::to_string(idx++), cin + feat.back(), cout});
      feat.pop_back();
      cin = cout;
    }
  }
  std::vector<LayerDesc> all;
  all.insert(all.end(), downs.begin(), downs.end());
  all.insert(all.end(), mid.begin(), mid.end());
  all.insert(all.end(), ups.begin(), ups.end());
  all.push_back({4, "final_conv", cout, c.out_channel});
  if (downs_out) *downs_out = downs;
  if (mid_out) *mid_out = mid;
  if (ups_out) *ups_out = ups;
  return all;
}

static std::map<std::string, std::vector<int64_t>> unet_param_shapes(const UNetCfg& c) {
  std::map<std::string, std::vector<int64_t>> s;
  const int64_t inner = c.inner;
  s["noise_level_mlp.1.weight"] = {inner * 4, inner};
  s["noise_level_mlp.1.bias"] = {inner * 4};
  s["noise_level_mlp.3.weight"] = {inner, inner * 4};
  s["noise_level_mlp.3.bias"] = {inner};
  for (const auto& L : unet_layers(c, nullptr, nullptr, nullptr)) {
    const std::string& n = L.name;
    if (L.kind == 1) {
      s[n + ".noise_func.noise_func.0.weight"] = {L.cout, inner};
      s[n + ".noise_func.noise_func.0.bias"] = {L.cout};
      s[n + ".block1.block.0.weight"] = {L.cin};
      s[n + ".block1.block.0.bias"] = {L.cin};
      s[n + ".block1.block.3.weight"] = {L.cout, L.cin, 3, 3};
      s[n + ".block1.block.3.bias"] = {L.cout};
      s[n + ".block2.block.0.weight"] = {L.cout};
      s[n + ".block2.block.0.bias"] = {L.cout};
      s[n + ".block2.block.3.weight"] = {L.cout, L.cout, 3, 3};
      s[n + ".block2.block.3.bias"] = {L.cout};
      if (L.cin != L.cout) {
        s[n + ".res_conv.weight"] = {L.cout, L.cin, 1, 1};
        s[n + ".res_conv.bias"] = {L.cout};
      }
    } else if (L.kind == 2 || L.kind == 3) {
      s[n + ".conv.weight"] = {L.cout, L.cin, 3, 3};
      s[n + ".conv.bias"] = {L.cout};
    } else if (L.kind == 0) {
      s[n + ".weight"] = {L.cout, L.cin, 3, 3};
      s[n + ".bias"] = {L.cout};
    } else {
      s[n + ".block.0.weight"] = {L.cin};
      s[n + ".block.0.bias"] = {L.cin};
      s[n + ".block.3.weight"] = {L.cout, L.cin, 3, 3};
      s[n + ".block.3.bias"] = {L.cout};
    }
  }
  return s;
}

// ---------------------------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------------------------
struct Param { std::vector<int64_t> shape; std::vector<float> data; bool loaded = false; };
struct Tensor { void* p = nullptr; int C = 0, H = 0, W = 0; float* stats = nullptr; int tiles = 0, n_tile = 0; };
struct Op {
  int cls;  // 0 conv_in, 1 gn, 2 conv3x3, 3 final, 4 other
  double bytes, flops;
  std::function<hipError_t(hipStream_t)> run;
  std::string name = "";
  std::function<hipError_t(hipStream_t, int)> run_dbg = nullptr;   // ablation relaunch (timing experiments)
  std::string kname = "";   // kernel family the op launches (template arguments that pick the tiling)
  std::string kinst = "";   // the exact template instantiation (as rocprofv3 lists it), for per-kernel profiles
};
struct ProfAcc { double ms = 0; int64_t n = 0; double bytes = 0, flops = 0; };

struct RunState {  // fields patched into the plan's kernel arguments at launch time
  const float* cond = nullptr;
  float* x = nullptr;
  const float* temb = nullptr;
  int temb_per_b = 0;
  int* t_dev = nullptr;
  int final_mode = 0;
  float* eps_out = nullptr;
  uint64_t seed = 0;
  int64_t row_offset = 0;
  const float* noise = nullptr;   // caller-supplied draws of this lane's rows (sddm_sample_noise), or null
  int64_t noise_ld = 0;
};

static constexpr int kStreams = 4;    // concurrent lane streams (GPU_MAX_HW_QUEUES is 4)
static constexpr int kMaxLanes = 64;  // step counters reserved in the weight arena

struct Lane {                         // one row block of the batch: plan + activations + graph
  int B = 0, row0 = 0, idx = 0;
  Arena arena;
  std::vector<Op> ops;
  RunState rs;
  size_t off_temb_fwd = 0, off_cond = 0, off_x = 0;
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  int g_K = 0, g_gen = -1;
  ~Lane() {
    if (gexec) (void)hipGraphExecDestroy(gexec);
    if (graph) (void)hipGraphDestroy(graph);
    arena.reset();
  }
};

struct DWState;                       // DiffWave path (dw_runtime.h)
struct WGState;                       // WaveGrad path (wg_runtime.h)

struct sddm_ctx {
  int device = 0, dtype = DT_BF16;
  bool configured = false;
  // arch / diffusion
  std::string arch_type, net_type, p_transition = "original";
  int noise_time_step = 0;
  int tr_mode = SDDM_TR_ORIGINAL, init_mode = 0;
  int T = 0, num_samples = -1;
  std::vector<float> tables;  // [14][T+1]
  bool tables_dirty = true;
  UNetCfg ucfg;
  std::map<std::string, Param> params;
  bool params_dirty = true;
  // device state
  Arena warena;      // weights + tables + temb table
  size_t off_tables = 0, off_tdev = 0, off_temb_tab = 0;
  std::map<std::string, size_t> woff;  // packed weight offsets
  int SC = 0;
  std::map<std::string, int> temb_off;  // per ResnetBlock offset in the projection vector
  // the batch is split into lanes of at most lane_rows rows; each lane has its own plan,
  // activations and step counter, and the lanes' step graphs are replayed concurrently on
  // kStreams streams (the deep UNet levels are latency-bound: independent lanes fill the chip)
  std::vector<std::unique_ptr<Lane>> lanes;
  int plan_B = -1;
  int lane_rows = 16;
  int plan_gen = 0;
  hipStream_t work[kStreams] = {};
  hipEvent_t ev_in = nullptr;
  hipEvent_t ev_done[kStreams] = {};
  bool use_graphs = true;
  // profiling
  unsigned long long* stamp_buf = nullptr;   // SDDM_STAMPS builds: phase stamps of one op
  int64_t stamp_blocks = 0;
  bool prof = false;
  // profiling (sddm_profile_enable): HIP events around every launch, drained after each step of
  // a lane into per-op accumulators, so every launch of a sampling run is timed with a small pool
  std::vector<hipEvent_t> ev_pool;
  std::vector<std::pair<int, int>> ev_pend;   // (op index, pool index of the start event)
  std::vector<ProfAcc> op_acc;                // per op index (the same layer list in every lane)
  // SDDM_spectrogram + DiffWave
  std::shared_ptr<DWState> dws;
  std::shared_ptr<WGState> wgs;
  // measured per-layer kernel tables (sddm_set_conv_tuning), each valid for one lane batch /
  // dtype / num_samples: conv_deep tiles per layer name (pixels per block, waves) and the kernel
  // choice (1 strip, 2 tile (a = configuration), 3 deep (a = pixels, b = waves, c = channels))
  struct KernTune { int kind, a, b, c; };
  struct TuneTable {
    std::map<std::string, std::pair<int, int>> deep_tune;
    std::map<std::string, KernTune> kern_tune;
    int B = -1, dtype = -1, N = -1;
  };
  std::vector<TuneTable> tunes;
  int hop_samples = 256;

  const float* dtab(int k) const { return warena.at<float>(off_tables) + (size_t)k * (T + 1); }
  TransCoef coef() const {
    TransCoef c;
    c.betas = dtab(0); c.alphas = dtab(1); c.sqrt_alpha_bar = dtab(3); c.pnc = dtab(4);
    c.sigma = dtab(5); c.sgamma = dtab(6); c.ssh = dtab(7); c.sqrt_delta = dtab(9);
    c.c_xt = dtab(10); c.c_yt = dtab(11); c.c_epst = dtab(12); c.sde = dtab(13);
    return c;
  }
};

// ---------------------------------------------------------------------------------------------
// weight upload: pack every layer into the kernels' layouts in the compute dtype
// ---------------------------------------------------------------------------------------------
static int upload_weights(sddm_ctx* c) {
  const int dt = c->dtype;
  const size_t es = dtype_size(dt);
  auto P = [&](const std::string& k) -> const Param& { return c->params.at(k); };
  c->warena.reset();
  c->woff.clear();
  c->temb_off.clear();
  Arena& A = c->warena;
  struct Blob { size_t off; std::vector<char> bytes; };
  std::vector<Blob> blobs;
  auto add_f32 = [&](const std::string& name, const std::vector<float>& v) {
    Blob b;
    b.bytes.resize(v.size() * 4);
    std::memcpy(b.bytes.data(), v.data(), b.bytes.size());
    b.off = A.reserve(b.bytes.size());
    c->woff[name] = b.off;
    blobs.push_back(std::move(b));
  };
  // 3x3 conv weight [co][ci][3][3] -> [co_pad64][ci/32][9][32] (T)
  auto add_conv3 = [&](const std::string& name, const Param& w) {
    const int co = (int)w.shape[0], ci = (int)w.shape[1];
    const int cop = (co + 63) / 64 * 64, nch = ci / 32;
    Blob b;
    b.bytes.assign((size_t)cop * ci * 9 * es, 0);
    for (int o = 0; o < co; ++o)
      for (int i = 0; i < ci; ++i)
        for (int tap = 0; tap < 9; ++tap) {
          const size_t dst = (((size_t)o * nch + i / 32) * 9 + tap) * 32 + (i % 32);
          store_elem(b.bytes.data(), dst, w.data[((size_t)o * ci + i) * 9 + tap], dt);
        }
    b.off = A.reserve(b.bytes.size());
    c->woff[name] = b.off;
    blobs.push_back(std::move(b));
    {  // conv_deep fragment image [co/16][ci/32 * 9][64 lanes][8]: lane l of step s holds
       // W[16 cb + (l & 15)][32 (s / 9) + 8 (l >> 4) + j][tap s % 9]
      Blob bf;
      const int ns = (ci / 32) * 9;
      bf.bytes.assign((size_t)co * ci * 9 * es, 0);
      for (int o = 0; o < co; ++o)
        for (int i = 0; i < ci; ++i)
          for (int tap = 0; tap < 9; ++tap) {
            const int s = (i / 32) * 9 + tap, l = (o % 16) + 16 * ((i % 32) / 8);
            const size_t dst = (((size_t)(o / 16) * ns + s) * 64 + l) * 8 + i % 8;
            store_elem(bf.bytes.data(), dst, w.data[((size_t)o * ci + i) * 9 + tap], dt);
          }
      bf.off = A.reserve(bf.bytes.size());
      c->woff[name + "_f"] = bf.off;
      blobs.push_back(std::move(bf));
    }
    if (dt != DT_F32) {  // conv_tile image [ci/32][9][4][co][8]: one 16-byte unit = 8 input channels
      Blob bt;
      bt.bytes.assign((size_t)co * ci * 9 * es, 0);
      for (int o = 0; o < co; ++o)
        for (int i = 0; i < ci; ++i)
          for (int tap = 0; tap < 9; ++tap) {
            const size_t dst = ((((size_t)(i / 32) * 9 + tap) * 4 + (i % 32) / 8) * co + o) * 8 + i % 8;
            store_elem(bt.bytes.data(), dst, w.data[((size_t)o * ci + i) * 9 + tap], dt);
          }
      bt.off = A.reserve(bt.bytes.size());
      c->woff[name + "_t"] = bt.off;
      blobs.push_back(std::move(bt));
    }
  };
  auto add_conv1 = [&](const std::string& name, const Param& w) {  // [co][ci] -> [co_pad64][ci]
    const int co = (int)w.shape[0], ci = (int)w.shape[1];
    const int cop = (co + 63) / 64 * 64;
    Blob b;
    b.bytes.assign((size_t)cop * ci * es, 0);
    for (int o = 0; o < co; ++o)
      for (int i = 0; i < ci; ++i) store_elem(b.bytes.data(), (size_t)o * ci + i, w.data[(size_t)o * ci + i], dt);
    b.off = A.reserve(b.bytes.size());
    c->woff[name] = b.off;
    blobs.push_back(std::move(b));
    {  // conv_deep fragment image [co/16][ci/32][64 lanes][8]
      Blob bf;
      bf.bytes.assign((size_t)co * ci * es, 0);
      for (int o = 0; o < co; ++o)
        for (int i = 0; i < ci; ++i) {
          const int l = (o % 16) + 16 * ((i % 32) / 8);
          store_elem(bf.bytes.data(), (((size_t)(o / 16) * (ci / 32) + i / 32) * 64 + l) * 8 + i % 8,
                     w.data[(size_t)o * ci + i], dt);
        }
      bf.off = A.reserve(bf.bytes.size());
      c->woff[name + "_f"] = bf.off;
      blobs.push_back(std::move(bf));
    }
    if (dt != DT_F32) {  // conv_tile image [ci/32][4][co][8]
      Blob bt;
      bt.bytes.assign((size_t)co * ci * es, 0);
      for (int o = 0; o < co; ++o)
        for (int i = 0; i < ci; ++i)
          store_elem(bt.bytes.data(), (((size_t)(i / 32) * 4 + (i % 32) / 8) * co + o) * 8 + i % 8,
                     w.data[(size_t)o * ci + i], dt);
      bt.off = A.reserve(bt.bytes.size());
      c->woff[name + "_t"] = bt.off;
      blobs.push_back(std::move(bt));
    }
  };
  const std::string pfx = "";
  std::vector<float> pw, pb;
  int sc = 0;
  for (const auto& L : unet_layers(c->ucfg, nullptr, nullptr, nullptr)) {
    const std::string& n = L.name;
    if (L.kind == 0) {
      add_f32(n + ".weight", P(n + ".weight").data);
      add_f32(n + ".bias", P(n + ".bias").data);
    } else if (L.kind == 1) {
      add_f32(n + ".block1.gamma", P(n + ".block1.block.0.weight").data);
      add_f32(n + ".block1.beta", P(n + ".block1.block.0.bias").data);
      add_conv3(n + ".block1.w", P(n + ".block1.block.3.weight"));
      add_f32(n + ".block1.b", P(n + ".block1.block.3.bias").data);
      add_f32(n + ".block2.gamma", P(n + ".block2.block.0.weight").data);
      add_f32(n + ".block2.beta", P(n + ".block2.block.0.bias").data);
      add_conv3(n + ".block2.w", P(n + ".block2.block.3.weight"));
      std::vector<float> b2 = P(n + ".block2.block.3.bias").data;
      if (L.cin != L.cout) {
        add_conv1(n + ".res.w", P(n + ".res_conv.weight"));
        const auto& rb = P(n + ".res_conv.bias").data;
        for (int i = 0; i < L.cout; ++i) b2[i] = b2[i] + rb[i];
      }
      add_f32(n + ".block2.b", b2);
      const auto& fw = P(n + ".noise_func.noise_func.0.weight").data;
      const auto& fb = P(n + ".noise_func.noise_func.0.bias").data;
      pw.insert(pw.end(), fw.begin(), fw.end());
      pb.insert(pb.end(), fb.begin(), fb.end());
      c->temb_off[n] = sc;
      sc += L.cout;
    } else if (L.kind == 2 || L.kind == 3) {
      add_conv3(n + ".w", P(n + ".conv.weight"));
      add_f32(n + ".b", P(n + ".conv.bias").data);
    } else {
      add_f32(n + ".gamma", P(n + ".block.0.weight").data);
      add_f32(n + ".beta", P(n + ".block.0.bias").data);
      add_f32(n + ".w", P(n + ".block.3.weight").data);  // [1][C][3][3]
      add_f32(n + ".b", P(n + ".block.3.bias").data);
    }
  }
  add_f32("mlp.w1", P("noise_level_mlp.1.weight").data);
  add_f32("mlp.b1", P("noise_level_mlp.1.bias").data);
  add_f32("mlp.w2", P("noise_level_mlp.3.weight").data);
  add_f32("mlp.b2", P("noise_level_mlp.3.bias").data);
  add_f32("proj.w", pw);
  add_f32("proj.b", pb);
  {  // PositionalEncoding.embedding_vector (UNetModified2.py:53-55), fp32 ops as torch
    const int half = c->ucfg.inner / 2;
    std::vector<float> ev(half);
    for (int k = 0; k < half; ++k) {
      const float e = (-(float)k * 4.0f) / (float)half;
      ev[k] = 1e4f * std::pow(10.0f, e);
    }
    add_f32("emb_vec", ev);
  }
  c->SC = sc;
  c->off_tables = A.reserve(sizeof(float) * 14 * (c->T + 1));
  c->off_tdev = A.reserve(64 * kMaxLanes);
  c->off_temb_tab = A.reserve(sizeof(float) * (size_t)(c->T + 1) * sc);
  SDDM_HIP_CHECK(A.commit());
  for (const auto& b : blobs) SDDM_HIP_CHECK(hipMemcpy(A.base + b.off, b.bytes.data(), b.bytes.size(), hipMemcpyHostToDevice));
  c->params_dirty = false;
  c->tables_dirty = true;
  c->plan_B = -1;  // plans hold weight pointers
  return SDDM_OK;
}

static int upload_tables(sddm_ctx* c) {
  SDDM_HIP_CHECK(hipMemcpy(c->warena.base + c->off_tables, c->tables.data(), sizeof(float) * c->tables.size(),
                           hipMemcpyHostToDevice));
  c->tables_dirty = false;
  return SDDM_OK;
}

#include "dw_runtime.h"
#include "wg_runtime.h"

// ---------------------------------------------------------------------------------------------
// plan: the launch sequence of one UNetModified2 step for batch B
// ---------------------------------------------------------------------------------------------
struct ConvChoice {
  int strip = 0;      // 1: row-streaming kernel (conv_strip.hip), 0: whole-K tile kernel (conv_deep.hip)
  int nblk = 32, SR = 0, mpi = 128;
  int mt = 0, ckb = 0, nw = 4, nb = 32;           // conv_deep: pixels per block, input chunks, waves, channels
  int tile = -1;                                  // conv_tile configuration (16-bit dtypes), -1: none
  int TR = 0, TW = 0, tiles_x = 0, n_tiles = 0;  // stats tiling of the output
  int chain = 0;                                  // 1: part of the bottom-level chain launch (conv_chain.hip)
};

// conv_deep tile (pixels per block) and waves per block.  A block's time is dominated by its
// one memory round trip, so the grid should need as few rounds of resident blocks as possible
// (256 CUs x 2 blocks at 4 waves, x 1 block at 8 waves); among equal round counts 8 waves (the
// K split 8 ways, weights resident) and then the smaller tile (less work per block) win.
// SDDM_DEEP_CFG=mt:nw forces one configuration wherever it fits (experiments).
static bool choose_deep(int dt, int B, ConvArgs a, bool s2, ConvChoice& ch, int want_mt = 0, int want_nw = 0,
                        int want_nb = 0) {
  static int force_mt = -1, force_nw = -1, force_nb = 0;
  if (force_mt < 0) {
    force_mt = force_nw = 0;
    if (const char* e = std::getenv("SDDM_DEEP_CFG")) std::sscanf(e, "%d:%d:%d", &force_mt, &force_nw, &force_nb);
  }
  // 16-channel blocks only where asked for (tuning table or SDDM_DEEP_CFG): twice the blocks, each
  // with half the weight bytes (the per-CU load volume bounds these layers) but the input halo
  // transformed twice as often
  // (a forced block width that does not divide a layer's channels leaves that layer at 32)
  const int nb = want_mt ? (want_nb ? want_nb : 32) : (force_nb && a.Cout % force_nb == 0 ? force_nb : 32);
  if (a.Cout % nb) return false;
  const int nz = a.Cout / nb;
  a.deep_nb = nb;
  struct Cand { int mt, nw, TR, TW, tiles_x, n_tiles, blocks, rounds; };
  std::vector<Cand> cs;
  for (int mt : {128, 64, 32, 16}) {
    if (mt == 16 && nb != 16) continue;
    const int TW = std::min(a.Wo, mt);
    if (mt % TW || a.Wo % TW) continue;
    const int TR = std::min(mt / TW, a.Ho);
    if (a.Ho % TR) continue;
    if (TR * TW < mt && mt > 32) continue;        // partial tiles only at the smallest size
    a.TR = TR; a.TW = TW; a.tiles_x = a.Wo / TW; a.n_tiles = a.tiles_x * (a.Ho / TR);
    for (int nw : {8, 4}) {
      a.deep_nw = nw;
      if (conv_deep_lds_bytes(dt, mt, s2, a) > kLdsBytes) continue;
      const int blocks = a.n_tiles * B * nz, per_round = 256 * (nw == 4 ? 2 : 1);
      cs.push_back({mt, nw, TR, TW, a.tiles_x, a.n_tiles, blocks, (blocks + per_round - 1) / per_round});
    }
  }
  if (cs.empty()) return false;
  const Cand* pick = nullptr;
  const int fm = want_mt ? want_mt : force_mt, fn = want_mt ? want_nw : force_nw;
  for (const Cand& c : cs)
    if (c.mt == fm && c.nw == fn) pick = &c;
  if (!pick) {
    pick = &cs[0];
    for (const Cand& c : cs) {
      if (c.rounds != pick->rounds) { if (c.rounds < pick->rounds) pick = &c; continue; }
      if (c.nw != pick->nw) { if (c.nw > pick->nw) pick = &c; continue; }
      if (c.mt < pick->mt) pick = &c;
    }
  }
  ch.strip = 0; ch.mt = pick->mt; ch.nw = pick->nw; ch.nb = nb; ch.ckb = (a.CA + a.CB) / 32;
  ch.TR = pick->TR; ch.TW = pick->TW; ch.tiles_x = pick->tiles_x; ch.n_tiles = pick->n_tiles;
  return true;
}

// conv_tile configuration: the largest pixel x channel tile (most reuse of each transformed input
// element and weight) among those whose grid still fills the chip; when no tile reaches 256
// blocks, the one with the most blocks.  SDDM_TILE_CFG=<i> forces configuration i wherever it
// fits; SDDM_NO_TILE=1 keeps every 16-bit layer on conv_deep (experiments).
// conv_deep block order: a tile's channel blocks on one XCD (the input halo read once per XCD,
// every XCD reading every weight slice) when the layer's input is at least its weights, else
// z-major (each XCD its own weight slices; the 8x4 / 16x8 levels, where weights dominate).  PMC:
// deep-level traffic 200.6 MB (z-major everywhere) -> 138.6 (channel-inner everywhere) -> ~130 MB
// per step.  SDDM_DEEP_ZIN=0/1 forces one order (A/B runs).
static int deep_zin(const ConvArgs& a, int B, size_t es) {
  static const int force = std::getenv("SDDM_DEEP_ZIN") ? std::atoi(std::getenv("SDDM_DEEP_ZIN")) : -1;
  if (force >= 0) return force;
  const double in = (double)B * a.Hi * a.Wi * (a.CA + a.CB) * es;
  const double w = (double)a.Cout * ((a.CA + a.CB) * 9 + (a.res_mode == 2 ? a.RCA + a.RCB : 0)) * es;
  return in >= w ? 1 : 0;
}

static bool choose_tile(int dt, int B, ConvArgs a, bool s2, ConvChoice& ch, int want = -1) {
  if (dt == DT_F32) return false;
  static const int force = std::getenv("SDDM_TILE_CFG") ? std::atoi(std::getenv("SDDM_TILE_CFG")) : -1;
  static const bool off = std::getenv("SDDM_NO_TILE") != nullptr;
  if (off) return false;
  const int fw = want >= 0 ? want : force;
  struct Cand { int cfg, TR, TW, tiles_x, n_tiles, blocks, area; };
  std::vector<Cand> cs;
  for (int cfg = 0; cfg < conv_tile_ncfg(); ++cfg) {
    const TileCfg t = conv_tile_cfg(cfg);
    const int MT = t.wpx * t.fp * 16, NB = t.wco * t.fc * 16;
    if (a.Cout % NB) continue;
    const int TW = std::min(a.Wo, MT);
    if (MT % TW || a.Wo % TW) continue;
    const int TR = std::min(MT / TW, a.Ho);
    if (a.Ho % TR) continue;
    if (TR * TW < MT && (TR != a.Ho || TW != a.Wo)) continue;   // partial tiles: whole small images only
    a.TR = TR; a.TW = TW; a.tiles_x = a.Wo / TW; a.n_tiles = a.tiles_x * (a.Ho / TR);
    if (conv_tile_lds_bytes(cfg, s2, a) > kLdsBytes) continue;
    cs.push_back({cfg, TR, TW, a.tiles_x, a.n_tiles, a.n_tiles * B * (a.Cout / NB), TR * TW * NB});
  }
  if (cs.empty()) return false;
  const Cand* pick = nullptr;
  for (const Cand& c : cs)
    if (c.cfg == fw) pick = &c;
  if (!pick) {
    for (const Cand& c : cs) {
      if (!pick) { pick = &c; continue; }
      const bool cf = c.blocks >= 256, pf = pick->blocks >= 256;
      if (cf != pf) { if (cf) pick = &c; continue; }
      if (!cf) { if (c.blocks != pick->blocks) { if (c.blocks > pick->blocks) pick = &c; continue; } }
      if (c.area > pick->area) pick = &c;
    }
  }
  ch.strip = 0; ch.tile = pick->cfg;
  ch.TR = pick->TR; ch.TW = pick->TW; ch.tiles_x = pick->tiles_x; ch.n_tiles = pick->n_tiles;
  return true;
}

static bool choose_conv(int dt, int B, int Cin, int RC, int res_mode, int Ho, int Wo, int Cout, bool s2, bool up,
                        ConvChoice& ch, int want_mt = 0, int want_nw = 0, int kind = 0, int ka = 0, int want_nb = 0) {
  ConvArgs a{};
  a.CA = Cin; a.CB = 0; a.RCA = RC; a.RCB = 0; a.res_mode = res_mode; a.Ho = Ho; a.Wo = Wo; a.Cout = Cout;
  a.upsample = up ? 1 : 0;
  a.Hi = up ? Ho / 2 : (s2 ? Ho * 2 : Ho); a.Wi = up ? Wo / 2 : (s2 ? Wo * 2 : Wo);
  // tuning knobs for experiments (unset = defaults): SDDM_STRIP_MPI=128|256, SDDM_STRIP_BLOCKS=target grid
  static const int env_mpi = std::getenv("SDDM_STRIP_MPI") ? std::atoi(std::getenv("SDDM_STRIP_MPI")) : 0;
  static const int env_blocks = std::getenv("SDDM_STRIP_BLOCKS") ? std::atoi(std::getenv("SDDM_STRIP_BLOCKS")) : 0;
  if (kind == 2) {
    ConvChoice t = ch;
    if (choose_tile(dt, B, a, s2, t, ka) && t.tile == ka) { ch = t; return true; }
  }
  if (!s2 && (Wo == 128 || Wo == 64) && std::getenv("SDDM_NO_STRIP") == nullptr && (kind == 0 || kind == 1)) {
    const int nbs[2] = {(Cout % 64 == 0) ? 64 : 32, 32};
    for (int mpi : {256, 128}) {
      if (env_mpi && mpi != env_mpi) continue;
      const int TRs = mpi / Wo;
      if (Ho % TRs) continue;
      for (int ni = 0; ni < 2; ++ni) {
        const int nb = nbs[ni];
        if (conv_strip_lds_bytes(dt, nb, mpi, a) > kLdsBytes) continue;
        const int nz = (Cout + nb - 1) / nb;
        int SR = 0;
        const int target = env_blocks ? env_blocks : 256;
        for (int m = 32; m >= 2; m /= 2) {   // longest strip that still gives >= target blocks
          const int sr = TRs * m;
          if (Ho % sr) continue;
          SR = sr;
          if ((Ho / sr) * B * nz >= target) break;
        }
        if (SR == 0) continue;
        ch.strip = 1; ch.nblk = nb; ch.SR = SR; ch.mpi = mpi;
        ch.TR = SR; ch.TW = Wo; ch.tiles_x = 1; ch.n_tiles = Ho / SR;
        return true;
      }
    }
  }
  if (want_mt == 0 && kind != 3 && choose_tile(dt, B, a, s2, ch)) return true;
  return choose_deep(dt, B, a, s2, ch, want_mt, want_nw, want_nb);
}

static int build_lane(sddm_ctx* c, Lane& L) {
  const int B = L.B;
  Lane* lp = &L;
  const int dt = c->dtype;
  const size_t es = dtype_size(dt);
  const UNetCfg& u = c->ucfg;
  const int N = c->num_samples, W = u.seg, S = u.stride;
  const int F = (N - W) / S + 1;
  L.ops.clear();
  L.arena.reset();
  Arena& A = L.arena;

  // ---- pass 1: symbolic program + buffer reservations ----
  struct TRes { size_t p, st; int C, H, W, tiles, n_tile; };
  std::vector<TRes> tres;
  auto new_tensor = [&](int C, int H, int Wd, int tiles, int n_tile) -> int {
    TRes t;
    t.p = A.reserve((size_t)B * H * Wd * C * es);
    t.st = A.reserve(sizeof(float) * (size_t)B * tiles * C * 2);
    t.C = C; t.H = H; t.W = Wd; t.tiles = tiles; t.n_tile = n_tile;
    tres.push_back(t);
    return (int)tres.size() - 1;
  };
  struct GNRes { int a, b; std::string w; };   // GroupNorm sources (finalized in the consumer)
  std::vector<GNRes> gres;
  auto new_gn = [&](int xa, int xb, const std::string& w) -> int {
    gres.push_back({xa, xb, w});
    return (int)gres.size() - 1;
  };
  L.off_temb_fwd = A.reserve(sizeof(float) * (size_t)B * std::max(c->SC, 1));
  L.off_cond = A.reserve(sizeof(float) * (size_t)B * N);
  L.off_x = A.reserve(sizeof(float) * (size_t)B * N);

  enum { ST_CONVIN, ST_GN, ST_CONV, ST_FINAL };
  struct Step {
    int type = 0;
    std::string w;          // weight-name prefix
    std::string rb;         // ResnetBlock name (temb offset / res weights), "" if none
    int srcA = -1, srcB = -1, gn = -1, out = -1;
    int s2 = 0, up = 0, res_mode = 0, rawA = -1, rawB = -1, cout = 0;
    bool temb = false;
    ConvChoice ch;
  };
  std::vector<Step> prog;
  // measured per-layer deep tiles (sddm_set_conv_tuning) apply when they were measured for this
  // lane batch, dtype and length; otherwise the round-count heuristic of choose_deep decides
  // kernel choices depend on the geometry and the lane capacity, never on the rows a lane holds:
  // every lane, and every row partition of a batch (sharded runs), gets the same kernels, tiles
  // and GroupNorm tilings, hence bit-identical rows
  const int PB = std::max(1, c->lane_rows);
  // A table measured for this exact dtype wins; failing that, a bfloat16 table also serves float16
  // (the same kernels at the same bytes and MFMA rate).  Never the other way: the float16 rows
  // (config #5) have fp16-only compile-time shapes (ConvShape::f16only).
  const sddm_ctx::TuneTable* tuned = nullptr;
  for (const auto& tt : c->tunes)
    if (tt.B == PB && tt.N == N && tt.dtype == dt) { tuned = &tt; break; }
  if (!tuned && dt == DT_F16)
    for (const auto& tt : c->tunes)
      if (tt.B == PB && tt.N == N && tt.dtype == DT_BF16) { tuned = &tt; break; }
  auto pick = [&](const std::string& name, int Cin, int RC, int res_mode, int Ho, int Wo, int cout, bool s2, bool up,
                  ConvChoice& ch) {
    int wm = 0, wn = 0, wb = 0, kind = 0, ka = 0;
    if (tuned) {
      auto it = tuned->deep_tune.find(name);
      if (it != tuned->deep_tune.end()) { wm = it->second.first; wn = it->second.second; kind = 3; }
      auto kt = tuned->kern_tune.find(name);
      if (kt != tuned->kern_tune.end()) {
        kind = kt->second.kind; ka = kt->second.a;
        if (kind == 3) { wm = kt->second.a; wn = kt->second.b; wb = kt->second.c; }
      }
    }
    // "chain": the layer runs inside the bottom-level chain launch; its tensor keeps the tiling the
    // heuristic would give it (only the chain reads or writes it)
    const bool chain = kind == 4 && dt != DT_F32;
    if (kind == 4) kind = 0;
    const bool ok = choose_conv(dt, PB, Cin, RC, res_mode, Ho, Wo, cout, s2, up, ch, wm, wn, kind, ka, wb);
    ch.chain = chain ? 1 : 0;
    return ok;
  };
  const int TRin = 512 / W;
  if (u.inner != 32 || 512 % W || F % TRin || (TRin + 1) * S + W + 2 > 1024)
    FAIL(SDDM_ERR_NOT_IMPLEMENTED, "conv_in needs inner_channel 32 and segment_len dividing 512 (got %d, %d)", u.inner, W);
  const int t0 = new_tensor(u.inner, F, W, F / TRin, TRin * W);
  { Step st; st.type = ST_CONVIN; st.out = t0; prog.push_back(st); }

  auto res_block = [&](const std::string& n, int xa, int xb, int cin, int cout) -> int {
    const int H = tres[xa].H, Wd = tres[xa].W;
    ConvChoice c1, c2;
    if (!pick(n + ".block1", cin, 0, 0, H, Wd, cout, false, false, c1)) return -1;
    if (!pick(n + ".block2", cout, cin, cin != cout ? 2 : 1, H, Wd, cout, false, false, c2)) return -1;
    const int g1 = new_gn(xa, xb, n + ".block1");
    const int h = new_tensor(cout, H, Wd, c1.n_tiles, c1.TR * c1.TW);
    { Step st; st.type = ST_CONV; st.w = n + ".block1"; st.rb = n; st.srcA = xa; st.srcB = xb; st.gn = g1;
      st.out = h; st.cout = cout; st.temb = true; st.ch = c1; prog.push_back(st); }
    const int g2 = new_gn(h, -1, n + ".block2");
    const int o = new_tensor(cout, H, Wd, c2.n_tiles, c2.TR * c2.TW);
    { Step st; st.type = ST_CONV; st.w = n + ".block2"; st.rb = n; st.srcA = h; st.gn = g2; st.out = o;
      st.cout = cout; st.res_mode = cin != cout ? 2 : 1; st.rawA = xa; st.rawB = xb; st.ch = c2; prog.push_back(st); }
    return o;
  };
  std::vector<LayerDesc> downs, mid, ups;
  unet_layers(u, &downs, &mid, &ups);
  std::vector<int> feats{t0};
  int cur = t0;
  for (size_t i = 1; i < downs.size(); ++i) {
    const LayerDesc& L = downs[i];
    if (L.kind == 1) {
      cur = res_block(L.name, cur, -1, L.cin, L.cout);
    } else {
      if (tres[cur].H % 2 || tres[cur].W % 2) FAIL(SDDM_ERR_SHAPE, "odd size before %s", L.name.c_str());
      const int H = tres[cur].H / 2, Wd = tres[cur].W / 2;
      ConvChoice ch;
      if (!pick(L.name, tres[cur].C, 0, 0, H, Wd, L.cout, true, false, ch)) FAIL(SDDM_ERR_SHAPE, "no tile for %s", L.name.c_str());
      const int o = new_tensor(L.cout, H, Wd, ch.n_tiles, ch.TR * ch.TW);
      Step st; st.type = ST_CONV; st.w = L.name; st.srcA = cur; st.out = o; st.s2 = 1; st.cout = L.cout; st.ch = ch;
      prog.push_back(st);
      cur = o;
    }
    if (cur < 0) FAIL(SDDM_ERR_SHAPE, "no tile for %s", L.name.c_str());
    feats.push_back(cur);
  }
  for (const LayerDesc& L : mid) {
    cur = res_block(L.name, cur, -1, L.cin, L.cout);
    if (cur < 0) FAIL(SDDM_ERR_SHAPE, "no tile for %s", L.name.c_str());
  }
  for (const LayerDesc& L : ups) {
    if (L.kind == 1) {
      const int skip = feats.back();
      feats.pop_back();
      if (tres[skip].H != tres[cur].H || tres[skip].W != tres[cur].W)
        FAIL(SDDM_ERR_SHAPE, "skip/upsample size mismatch at %s (torch.cat would raise)", L.name.c_str());
      cur = res_block(L.name, cur, skip, L.cin, L.cout);
      if (cur < 0) FAIL(SDDM_ERR_SHAPE, "no tile for %s", L.name.c_str());
    } else {
      const int H = tres[cur].H * 2, Wd = tres[cur].W * 2;
      ConvChoice ch;
      if (!pick(L.name, tres[cur].C, 0, 0, H, Wd, L.cout, false, true, ch)) FAIL(SDDM_ERR_SHAPE, "no tile for %s", L.name.c_str());
      const int o = new_tensor(L.cout, H, Wd, ch.n_tiles, ch.TR * ch.TW);
      Step st; st.type = ST_CONV; st.w = L.name; st.srcA = cur; st.out = o; st.up = 1; st.cout = L.cout; st.ch = ch;
      prog.push_back(st);
      cur = o;
    }
  }
  const int gf = new_gn(cur, -1, "final_conv");
  { Step st; st.type = ST_FINAL; st.srcA = cur; st.gn = gf; prog.push_back(st); }

  SDDM_HIP_CHECK(A.commit());

  // ---- pass 2: materialise kernel arguments ----
  auto TT = [&](int i) {
    Tensor t;
    if (i < 0) return t;
    const TRes& r = tres[i];
    t.p = A.base + r.p; t.stats = A.at<float>(r.st); t.C = r.C; t.H = r.H; t.W = r.W;
    t.tiles = r.tiles; t.n_tile = r.n_tile;
    return t;
  };
  auto WF = [&](const std::string& k) { return c->warena.at<float>(c->woff.at(k)); };
  auto WV = [&](const std::string& k) { return (const void*)(c->warena.base + c->woff.at(k)); };
  // the kernel arguments of one conv step, its algorithmic bytes and FLOPs
  auto conv_args = [&](const Step& st, ConvArgs& a, double& bytes, double& flops) -> int {
    a = ConvArgs{};
    const Tensor sa = TT(st.srcA), sb = TT(st.srcB), o = TT(st.out);
    a.srcA = sa.p; a.srcB = sb.p; a.CA = sa.C; a.CB = sb.C;
    a.Hi = sa.H; a.Wi = sa.W; a.Ho = o.H; a.Wo = o.W; a.upsample = st.up;
    a.Cout = st.cout; a.out = o.p; a.stats = o.stats;
    if (st.gn >= 0) {
      const GNRes& gr = gres[st.gn];
      const Tensor ga = TT(gr.a), gb = TT(gr.b);
      a.gstA = ga.stats; a.gtilesA = ga.tiles; a.gntileA = ga.n_tile;
      a.gstB = gb.stats; a.gtilesB = gb.tiles; a.gntileB = gb.n_tile;
      a.gamma = WF(gr.w + ".gamma"); a.beta = WF(gr.w + ".beta"); a.groups = u.groups; a.eps = 1e-5f;
      const int Ct = ga.C + gb.C;
      if (Ct % u.groups || (gb.C && ga.C % (Ct / u.groups)) || 256 % u.groups)
        FAIL(SDDM_ERR_SHAPE, "GroupNorm(%d, %d) at %s: unsupported grouping", u.groups, Ct, gr.w.c_str());
    }
    a.wgt = WV(st.w + ".w"); a.bias = WF(st.w + ".b");
    a.wgt_t = c->woff.count(st.w + ".w_t") ? WV(st.w + ".w_t") : nullptr;
    a.wgt_f = WV(st.w + ".w_f");
    a.res_mode = st.res_mode;
    const int Cin = a.CA + a.CB;
    bytes = (double)B * a.Hi * a.Wi * Cin * es + (double)B * a.Ho * a.Wo * a.Cout * es +
            (double)a.Cout * 9 * Cin * es;
    flops = 2.0 * B * a.Ho * a.Wo * a.Cout * 9.0 * Cin;
    if (st.res_mode == 1) {
      a.res_src = TT(st.rawA).p;
      bytes += (double)B * a.Ho * a.Wo * a.Cout * es;
    } else if (st.res_mode == 2) {
      const Tensor ra = TT(st.rawA), rb = TT(st.rawB);
      a.rawA = ra.p; a.rawB = rb.p; a.RCA = ra.C; a.RCB = rb.C;
      a.res_wgt = WV(st.rb + ".res.w");
      a.res_wgt_t = c->woff.count(st.rb + ".res.w_t") ? WV(st.rb + ".res.w_t") : nullptr;
      a.res_wgt_f = WV(st.rb + ".res.w_f");
      if ((ra.C + rb.C) % 32) FAIL(SDDM_ERR_SHAPE, "%s.res_conv: channels must be multiples of 32", st.rb.c_str());
      bytes += (double)B * a.Ho * a.Wo * (ra.C + rb.C) * es + (double)a.Cout * (ra.C + rb.C) * es;
      flops += 2.0 * B * a.Ho * a.Wo * a.Cout * (double)(ra.C + rb.C);
    }
    const ConvChoice& ch = st.ch;
    a.TR = ch.TR; a.TW = ch.TW; a.tiles_x = ch.tiles_x; a.n_tiles = ch.n_tiles;
    if (a.n_tiles != o.tiles || a.TR * a.TW != o.n_tile) FAIL(SDDM_ERR_STATE, "tile mismatch for %s", st.w.c_str());
    if ((a.CA + a.CB) % 32 || a.Cout % 32) FAIL(SDDM_ERR_SHAPE, "%s: channels must be multiples of 32", st.w.c_str());
    return SDDM_OK;
  };
  sddm_ctx* ctx = c;
  for (size_t si = 0; si < prog.size(); ++si) {
    const Step& st = prog[si];
    if (st.type == ST_CONV && st.ch.chain) {
      // the bottom level in one launch (conv_chain.hip): the last Downsample and the four convs of
      // mid.0 and ups.0, every one marked "chain" in the tuning table
      if (si + 4 >= prog.size()) FAIL(SDDM_ERR_SHAPE, "chain: %s is not followed by mid.0 / ups.0", st.w.c_str());
      const Step* S5[5] = {&prog[si], &prog[si + 1], &prog[si + 2], &prog[si + 3], &prog[si + 4]};
      const char* want[5] = {nullptr, "mid.0.block1", "mid.0.block2", "ups.0.block1", "ups.0.block2"};
      for (int k = 0; k < 5; ++k)
        if (S5[k]->type != ST_CONV || !S5[k]->ch.chain || (k > 0 && S5[k]->w != want[k]) || (k == 0 && !S5[k]->s2))
          FAIL(SDDM_ERR_SHAPE, "chain: the tuning table must mark the last Downsample, mid.0.block1/2 and ups.0.block1/2 (got %s)",
               S5[k]->w.c_str());
      ConvArgs ca[5];
      double bytes = 0, flops = 0;
      for (int k = 0; k < 5; ++k) {
        double by = 0, fl = 0;
        if (const int r = conv_args(*S5[k], ca[k], by, fl)) return r;
        flops += fl;
      }
      const int Cc = ca[0].Cout, Hc = ca[0].Ho, Wc = ca[0].Wo;
      if (ca[1].CA != Cc || ca[3].CA != Cc || ca[3].CB != Cc || ca[4].res_mode != 2 || ca[4].RCA != Cc || ca[4].RCB != Cc ||
          ca[2].res_mode != 1 || ca[3].srcB != ca[0].out || ca[4].rawB != ca[0].out)
        FAIL(SDDM_ERR_SHAPE, "chain: unexpected bottom-level wiring");
      ChainArgs x{};
      x.x = ca[0].srcA; x.out = ca[4].out;
      for (int k = 0; k < 5; ++k) { x.wgt[k] = ca[k].wgt_f; x.bias[k] = ca[k].bias; }
      for (int k = 0; k < 4; ++k) { x.gamma[k] = ca[k + 1].gamma; x.beta[k] = ca[k + 1].beta; }
      x.res_wgt = ca[4].res_wgt_f;
      x.temb_ld = c->SC; x.C = Cc; x.H = Hc; x.W = Wc; x.groups = u.groups; x.eps = 1e-5f;
      bytes = (double)B * (2 * Hc) * (2 * Wc) * Cc * es + (double)B * Hc * Wc * Cc * es;
      for (int k = 0; k < 5; ++k) bytes += (double)ca[k].Cout * (ca[k].CA + ca[k].CB) * 9 * es;
      bytes += (double)Cc * 2 * Cc * es;
      const int toff_m = c->temb_off.at("mid.0"), toff_u = c->temb_off.at("ups.0");
      std::string nm;
      for (int k = 0; k < 5; ++k) nm += (k ? "+" : "") + S5[k]->w;
      L.ops.push_back({2, bytes, flops, [lp, x, dt, B, toff_m, toff_u](hipStream_t s) {
                          ChainArgs y = x;
                          y.temb[0] = lp->rs.temb ? lp->rs.temb + toff_m : nullptr;
                          y.temb[1] = lp->rs.temb ? lp->rs.temb + toff_u : nullptr;
                          y.temb_per_b = lp->rs.temb_per_b;
                          y.t_dev = lp->rs.t_dev;
                          return launch_conv_chain(dt, y, B, s);
                        }, nm + "[chain]"});
      char kn[96];
      snprintf(kn, sizeof(kn), "conv_chain_kernel<%s,%d,%d,%d>", dt_name(dt), Cc, Hc, Wc);
      L.ops.back().kname = kn;
      L.ops.back().kinst = kn;
      si += 4;
      continue;
    }
    if (st.type == ST_CONVIN) {
      ConvInArgs a{};
      a.N = N; a.F = F; a.W = W; a.S = S; a.Cout = u.inner;
      a.w = WF("downs.0.weight"); a.bias = WF("downs.0.bias");
      const Tensor o = TT(st.out);
      a.out = o.p; a.stats = o.stats; a.TR = TRin;
      const double bytes = (double)B * N * 4 * 2 + (double)B * F * W * u.inner * es;
      const double flops = 2.0 * B * F * W * u.inner * 18;
#ifdef SDDM_STAMPS
      if (const char* sn = std::getenv("SDDM_STAMPS"))
        if (std::string(sn) == "downs.0") {
          if (!c->stamp_buf) SDDM_HIP_CHECK(hipMalloc(&c->stamp_buf, sizeof(unsigned long long) * 8 * 65536));
          a.stamps = c->stamp_buf;
          c->stamp_blocks = (int64_t)(F / TRin) * B;
        }
#endif
      L.ops.push_back({0, bytes, flops, [lp, a, dt, B](hipStream_t s) {
                          ConvInArgs x = a;
                          x.cond = lp->rs.cond; x.x = lp->rs.x; x.t_dev = lp->rs.t_dev;
                          return launch_conv_in(dt, x, B, s);
                        }, "downs.0"});
      L.ops.back().kname = std::string("conv_in_kernel<") + dt_name(dt) + ">";
      L.ops.back().kinst = L.ops.back().kname;
    } else if (st.type == ST_CONV) {
      ConvArgs a;
      double bytes = 0, flops = 0;
      if (const int r = conv_args(st, a, bytes, flops)) return r;
      const int Cin = a.CA + a.CB;
      const ConvChoice ch = st.ch;
      const bool s2 = st.s2 != 0;
      const bool temb = st.temb;
      if (std::getenv("SDDM_PRINT_SHAPES"))   // rows for kTileShapes / kDeepShapes / kStripShapes
        fprintf(stderr, "SHAPE %s %s%d s2=%d TR=%d TW=%d Ho=%d Wo=%d CA=%d CB=%d Cout=%d RCA=%d RCB=%d res=%d gn=%d up=%d mt=%d nw=%d nb=%d nblk=%d mpi=%d SR=%d ntiles=%d\n",
                st.w.c_str(), ch.strip ? "strip" : (ch.tile >= 0 ? "tile" : "deep"), ch.tile >= 0 ? ch.tile : ch.mt, s2 ? 1 : 0,
                a.TR, a.TW, a.Ho, a.Wo, a.CA, a.CB, a.Cout, a.RCA, a.RCB, a.res_mode, a.gamma ? 1 : 0, a.upsample ? 1 : 0,
                ch.mt, ch.nw, ch.nb, ch.nblk, ch.mpi, ch.SR, a.n_tiles);
      const int toff = temb ? c->temb_off.at(st.rb) : 0;
#ifdef SDDM_STAMPS
      if (const char* sn = std::getenv("SDDM_STAMPS")) {
        if (st.w == sn) {
          if (!c->stamp_buf) SDDM_HIP_CHECK(hipMalloc(&c->stamp_buf, sizeof(unsigned long long) * 8 * 65536));
          SDDM_HIP_CHECK(hipMemset(c->stamp_buf, 0, sizeof(unsigned long long) * 8 * 65536));
          a.stamps = c->stamp_buf;
          if (const char* f = std::getenv("SDDM_STAMPS_DBG")) a.dbg = std::atoi(f);   // timing ablations
          int nb = 32;
          if (ch.tile >= 0) { const TileCfg tc = conv_tile_cfg(ch.tile); nb = tc.wco * tc.fc * 16; }
          c->stamp_blocks = ch.strip ? (int64_t)(a.Ho / ch.SR) * B * ((a.Cout + ch.nblk - 1) / ch.nblk)
                                     : (int64_t)a.n_tiles * B * (a.Cout / (ch.tile >= 0 ? nb : ch.nb));
        }
      }
#endif
      L.ops.push_back({2, bytes, flops, [ctx, lp, a, s2, ch, dt, B, temb, toff](hipStream_t s) {
                          ConvArgs x = a;
                          if (temb) {
                            x.temb = lp->rs.temb + toff;
                            x.temb_ld = ctx->SC;
                            x.temb_per_b = lp->rs.temb_per_b;
                            x.t_dev = lp->rs.t_dev;
                          }
                          if (ch.strip) return launch_conv_strip(dt, ch.nblk, ch.mpi, ch.SR, x, B, s);
                          if (ch.tile >= 0) return launch_conv_tile(dt, ch.tile, s2, x, B, s);
                          x.deep_zin = deep_zin(x, B, dtype_size(dt)); x.deep_nw = ch.nw; x.deep_nb = ch.nb;
                          return launch_conv_deep(dt, ch.mt, s2, x, B, s);
                        }, st.w + (ch.strip ? "[strip]" : (ch.tile >= 0 ? "[tile" + std::to_string(ch.tile) + "]"
                                                                         : "[deep" + std::to_string(ch.mt) + "_" + std::to_string(ch.nw) + "_" + std::to_string(ch.nb) + "]"))});
      {
        char kn[160];
        if (ch.strip)
          snprintf(kn, sizeof(kn), "conv_strip_kernel<%s,%d,%d,%d,%d>", dt_name(dt), ch.nblk / 16, a.Wo, Cin, ch.mpi);
        else if (ch.tile >= 0) {
          const TileCfg tc = conv_tile_cfg(ch.tile);
          snprintf(kn, sizeof(kn), "conv_tile_kernel<%s,%d,%d,%d,%d,%d> (tile%d)", dt_name(dt), s2 ? 1 : 0, tc.wpx, tc.wco,
                   tc.fp, tc.fc, ch.tile);
        } else
          snprintf(kn, sizeof(kn), "conv_deep_kernel<%s,%d,%d,%d,%d>", dt_name(dt), s2 ? 1 : 0, ch.mt, ch.nw, ch.nb);
        L.ops.back().kname = kn;
        // instantiation: the strip kernel's residual mode / GroupNorm and the deep kernel's weight
        // ring depth are template arguments the family name leaves out
        char ki[192];
        if (ch.strip)
          snprintf(ki, sizeof(ki), "conv_strip_kernel<%s,%d,%d,%d,%d,%d,%d>", dt_name(dt), ch.nblk / 16, a.Wo, Cin,
                   ch.mpi, a.res_mode, a.gamma ? 1 : 0);
        else if (ch.tile >= 0)
          snprintf(ki, sizeof(ki), "%s", kn);
        else
          snprintf(ki, sizeof(ki), "conv_deep_kernel<%s,%d,%d,%d,%d,%d>", dt_name(dt), s2 ? 1 : 0, ch.mt, ch.nw,
                   conv_deep_ring_depth(dt, ch.mt, ch.nw, (Cin / 32) * 9 + (a.res_mode == 2 ? (a.RCA + a.RCB) / 32 : 0), ch.nb),
                   ch.nb);
        L.ops.back().kinst = ki;
      }
      {  // flags: 1 no stats, 2 no GroupNorm transform, 4 no residual / embedding, 8 skip the K loop
        auto base = L.ops.back().run;
        ConvArgs a0 = a;
        L.ops.back().run_dbg = [lp, ctx, a0, s2, ch, dt, B, temb, toff](hipStream_t s, int fl) {
          ConvArgs x = a0;
          if (temb && !(fl & 4)) { x.temb = lp->rs.temb + toff; x.temb_ld = ctx->SC; x.temb_per_b = lp->rs.temb_per_b; x.t_dev = lp->rs.t_dev; }
          if (fl & 1) x.stats = nullptr;
          if (fl & 2) x.gamma = nullptr;
          if (fl & 4) x.res_mode = 0;
          x.dbg = fl;
          if (ch.strip) return launch_conv_strip(dt, ch.nblk, ch.mpi, ch.SR, x, B, s);
          if (ch.tile >= 0) return launch_conv_tile(dt, ch.tile, s2, x, B, s);
          x.deep_zin = deep_zin(x, B, dtype_size(dt)); x.deep_nw = ch.nw; x.deep_nb = ch.nb;
          return launch_conv_deep(dt, ch.mt, s2, x, B, s);
        };
        (void)base;
      }
    } else {
      FinalArgs f{};
      const Tensor src = TT(st.srcA);
      f.src = src.p; f.C = src.C;
      {
        const GNRes& gr = gres[st.gn];
        const Tensor ga = TT(gr.a);
        f.gst = ga.stats; f.gtiles = ga.tiles; f.gntile = ga.n_tile;
        f.gamma = WF("final_conv.gamma"); f.beta = WF("final_conv.beta"); f.groups = u.groups; f.eps = 1e-5f;
        if (ga.C % u.groups || 256 % u.groups) FAIL(SDDM_ERR_SHAPE, "final GroupNorm grouping");
      }
      f.w = WF("final_conv.w");
      f.bias = c->params.at("final_conv.block.3.bias").data[0];
      // frames per block: 8 (512 threads); SDDM_FINAL_FT=16 takes 16 (one 1024-thread block per CU,
      // 19 staged frame rows per 16 instead of 11 per 8: less halo re-read)
      static const int env_ft = std::getenv("SDDM_FINAL_FT") ? std::atoi(std::getenv("SDDM_FINAL_FT")) : 0;
      f.N = N; f.F = F; f.W = W; f.S = S; f.FT = (env_ft == 16 && F % 16 == 0) ? 16 : (F % 8 == 0 ? 8 : 2);
      if (F % f.FT || W % S) FAIL(SDDM_ERR_SHAPE, "final tile: frames %d, segment %d/%d", F, W, S);
      f.co = c->coef();
      const double bytes = (double)B * F * W * src.C * es + (double)B * N * 4 * 3;
      const double flops = 2.0 * B * F * W * src.C * 9;
#ifdef SDDM_STAMPS
      if (const char* sn = std::getenv("SDDM_STAMPS"))
        if (std::string(sn) == "final_conv") {
          if (!c->stamp_buf) SDDM_HIP_CHECK(hipMalloc(&c->stamp_buf, sizeof(unsigned long long) * 8 * 65536));
          f.stamps = c->stamp_buf;
          c->stamp_blocks = (int64_t)(F / f.FT) * B;
        }
#endif
      L.ops.push_back({3, bytes, flops, [lp, f, dt, B](hipStream_t s) {
                          FinalArgs x = f;
                          x.mode = lp->rs.final_mode; x.eps_out = lp->rs.eps_out;
                          x.x = lp->rs.x; x.cond = lp->rs.cond; x.t_dev = lp->rs.t_dev;
                          x.seed = lp->rs.seed; x.row_offset = lp->rs.row_offset;
                          x.noise = lp->rs.noise; x.noise_ld = lp->rs.noise_ld;
                          x.sp = lp->rs.t_dev ? (const StepParams*)lp->rs.t_dev : nullptr;
                          return launch_final(dt, x, B, s);
                        }, "final_conv"});
      L.ops.back().kname = std::string("final_kernel<") + dt_name(dt) + (f.FT >= 16 ? ",1024>" : ",512>");
      L.ops.back().kinst = L.ops.back().kname;
    }
  }
  return SDDM_OK;
}

// split the batch into lanes of lane_rows rows (the same per-lane plan for any row partition
// into multiples of lane_rows, so sharded runs stay bit-identical to a single run)
static int build_plan(sddm_ctx* c, int B) {
  c->lanes.clear();
  c->plan_B = -1;
  const int LR = std::max(1, c->lane_rows);
  const int nl = (B + LR - 1) / LR;
  if (nl > kMaxLanes) FAIL(SDDM_ERR_INVALID_ARG, "batch %d needs %d lanes (max %d): raise SDDM_LANE_ROWS", B, nl, kMaxLanes);
  for (int l = 0; l < nl; ++l) {
    std::unique_ptr<Lane> L(new Lane());
    L->idx = l;
    L->row0 = l * LR;
    L->B = std::min(LR, B - l * LR);
    const int r = build_lane(c, *L);
    if (r) { c->lanes.clear(); return r; }
    c->lanes.push_back(std::move(L));
  }
  c->plan_B = B;
  c->plan_gen++;
  return SDDM_OK;
}

// =============================================================================================
// C ABI
// =============================================================================================
static int ensure_ready(sddm_ctx* c) {
  if (!c || !c->configured) FAIL(SDDM_ERR_STATE, "context not configured");
  if (c->net_type.empty()) FAIL(SDDM_ERR_STATE, "context has no network (diffusion-only)");
  SDDM_HIP_CHECK(hipSetDevice(c->device));
  for (const auto& kv : c->params)
    if (!kv.second.loaded) FAIL(SDDM_ERR_STATE, "parameter %s not loaded", kv.first.c_str());
  if (c->params_dirty) {
    const int r = c->dws ? dw_upload_weights(c) : (c->wgs ? wg_upload_weights(c) : upload_weights(c));
    if (r) return r;
  }
  if (c->tables_dirty) {
    const int r = upload_tables(c);
    if (r) return r;
  }
  return SDDM_OK;
}

static int prof_drain(sddm_ctx* c, const Lane& L) {
  if (c->ev_pend.empty()) return SDDM_OK;
  SDDM_HIP_CHECK(hipEventSynchronize(c->ev_pool[c->ev_pend.back().second + 1]));
  if (c->op_acc.size() < L.ops.size()) c->op_acc.resize(L.ops.size());
  for (const auto& pe : c->ev_pend) {
    float m = 0;
    SDDM_HIP_CHECK(hipEventElapsedTime(&m, c->ev_pool[pe.second], c->ev_pool[pe.second + 1]));
    ProfAcc& a = c->op_acc[pe.first];
    a.ms += m; a.n += 1; a.bytes += L.ops[pe.first].bytes; a.flops += L.ops[pe.first].flops;
  }
  c->ev_pend.clear();
  return SDDM_OK;
}

static int run_ops(sddm_ctx* c, Lane& L, hipStream_t s) {
  for (const Op& op : L.ops) {
    const bool timed = c->prof && c->ev_pend.size() * 2 + 2 <= c->ev_pool.size();
    int e0 = 0;
    if (timed) {
      e0 = (int)c->ev_pend.size() * 2;
      SDDM_HIP_CHECK(hipEventRecord(c->ev_pool[e0], s));
    }
    hipError_t e = op.run(s);
    if (e != hipSuccess) FAIL(SDDM_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(e));
    {  // dev knob: SDDM_REPEAT_OP=<layer> SDDM_REPEAT_N=<n> relaunches one (idempotent) layer
      static const char* rop = std::getenv("SDDM_REPEAT_OP");
      static const int rn = std::getenv("SDDM_REPEAT_N") ? std::atoi(std::getenv("SDDM_REPEAT_N")) : 0;
      static const int rflags = std::getenv("SDDM_REPEAT_FLAGS") ? std::atoi(std::getenv("SDDM_REPEAT_FLAGS")) : 0;
      if (rop && op.name.rfind(rop, 0) == 0)
        for (int k = 0; k < rn && e == hipSuccess; ++k) e = (rflags && op.run_dbg) ? op.run_dbg(s, rflags) : op.run(s);
      if (e != hipSuccess) FAIL(SDDM_ERR_HIP, "kernel launch failed: %s", hipGetErrorString(e));
    }
    if (timed) {
      SDDM_HIP_CHECK(hipEventRecord(c->ev_pool[e0 + 1], s));
      c->ev_pend.push_back({(int)(&op - L.ops.data()), e0});
    }
  }
  if (c->prof) return prof_drain(c, L);
  return SDDM_OK;
}

extern "C" {

int sddm_abi_version(void) { return SDDM_ABI_VERSION; }
const char* sddm_last_error(void) { return g_last_error.c_str(); }

int sddm_create(int device, int compute_dtype, sddm_ctx** out) {
  if (!out) FAIL(SDDM_ERR_INVALID_ARG, "out is NULL");
  if (compute_dtype < 0 || compute_dtype > 2) FAIL(SDDM_ERR_INVALID_ARG, "bad dtype %d", compute_dtype);
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
    FAIL(SDDM_ERR_HIP, "no HIP device %d (count %d)", device, n);
  int lds = 0;
  if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess || lds < kLdsBytes)
    FAIL(SDDM_ERR_HIP, "device %d offers %d bytes of LDS per workgroup; the kernels are planned for %d (gfx950)", device,
         lds, kLdsBytes);
  sddm_ctx* c = new sddm_ctx();
  c->device = device;
  c->dtype = compute_dtype;
  c->use_graphs = std::getenv("SDDM_NO_GRAPH") == nullptr;
  if (const char* lr = std::getenv("SDDM_LANE_ROWS")) c->lane_rows = std::max(1, std::atoi(lr));
  *out = c;
  return SDDM_OK;
}

void sddm_destroy(sddm_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  for (int k = 0; k < kStreams; ++k) {
    if (c->work[k]) { (void)hipStreamSynchronize(c->work[k]); (void)hipStreamDestroy(c->work[k]); }
    if (c->ev_done[k]) (void)hipEventDestroy(c->ev_done[k]);
  }
  c->lanes.clear();
  if (c->dws) c->dws->act.reset();
  if (c->wgs) c->wgs->act.reset();
  if (c->ev_in) (void)hipEventDestroy(c->ev_in);
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  c->warena.reset();
  delete c;
}

int sddm_schedule(const char* schedule, int n_timestep, double linear_start, double linear_end, float* out) {
  if (!schedule || !out || n_timestep < 1) FAIL(SDDM_ERR_INVALID_ARG, "bad schedule arguments");
  if (compute_schedule(schedule, n_timestep, linear_start, linear_end, out))
    FAIL(SDDM_ERR_NOT_IMPLEMENTED, "schedule '%s'", schedule);
  return SDDM_OK;
}

int sddm_configure(sddm_ctx* c, const char* json) {
  if (!c || !json) FAIL(SDDM_ERR_INVALID_ARG, "NULL argument");
  Json cfg;
  try {
    cfg = Json::parse(json);
  } catch (const std::exception& e) {
    FAIL(SDDM_ERR_INVALID_ARG, "config JSON: %s", e.what());
  }
  const Json& arch = cfg.at("arch");
  const Json& diff = cfg.at("diffusion");
  const Json& net = cfg.at("network");
  c->arch_type = arch.string("type", "SDDM");
  // rows per lane ("lane_rows", default 16; SDDM_LANE_ROWS overrides).  Every lane's kernels are
  // chosen for lane_rows rows, so any row partition samples bit-identically; larger lanes give the
  // latency-bound deep levels bigger grids for large per-GPU batches (config #5, B=128 per GPU:
  // lanes of 64 sample 1.18x faster than lanes of 16) but grids sized for 64 rows underfill a
  // 16-row batch (the config #2 headline ran 0.62x as fast on them)
  if (!std::getenv("SDDM_LANE_ROWS")) {
    const int lr = (int)cfg.number("lane_rows", 16);
    if (lr < 1) FAIL(SDDM_ERR_INVALID_ARG, "lane_rows %d", lr);
    c->lane_rows = lr;
    c->plan_B = -1;
  }
  const Json& aa = arch.at("args");
  const std::string nc = aa.string("noise_condition", "sqrt_alpha_bar");
  if (nc != "sqrt_alpha_bar" && nc != "time_step") FAIL(SDDM_ERR_NOT_IMPLEMENTED, "noise_condition '%s'", nc.c_str());
  c->noise_time_step = nc == "time_step";
  if (c->arch_type == "SDDM") {
    const std::string pt = aa.string("p_transition", "original");
    const std::string qt = aa.string("q_transition", "original");
    if (pt == "original") { c->tr_mode = SDDM_TR_ORIGINAL; c->init_mode = 0; }
    else if (pt == "condition_in") { c->tr_mode = SDDM_TR_ORIGINAL; c->init_mode = 4; }
    else if (pt == "sr3") { c->tr_mode = SDDM_TR_SR3; c->init_mode = 1; }
    else if (pt == "supportive") { c->tr_mode = SDDM_TR_SUPPORTIVE; c->init_mode = 2; }
    else if (pt == "conditional") { c->tr_mode = SDDM_TR_CONDITIONAL; c->init_mode = 3; }
    else FAIL(SDDM_ERR_NOT_IMPLEMENTED, "p_transition '%s' (model.py:20-23)", pt.c_str());
    if (qt != "original" && qt != "conditional") FAIL(SDDM_ERR_NOT_IMPLEMENTED, "q_transition '%s'", qt.c_str());
    c->p_transition = pt;
  } else if (c->arch_type == "SDDM_spectrogram") {              // model.py:206-257
    c->tr_mode = SDDM_TR_ORIGINAL;
    c->init_mode = 0;
    c->p_transition = "original";
    c->hop_samples = (int)aa.number("hop_samples", 256);          // SURVEY Q6 default
    if (c->hop_samples < 1) FAIL(SDDM_ERR_INVALID_ARG, "hop_samples %d", c->hop_samples);
  } else {
    FAIL(SDDM_ERR_NOT_IMPLEMENTED, "arch type '%s'", c->arch_type.c_str());
  }
  if (diff.string("type", "GaussianDiffusion") != "GaussianDiffusion")
    FAIL(SDDM_ERR_NOT_IMPLEMENTED, "diffusion type '%s'", diff.string("type", "").c_str());
  const Json& da = diff.at("args");
  const std::string sched = da.string("schedule", "linear");
  const int T = (int)da.number("n_timestep", 1000);
  const double ls = da.number("linear_start", 1e-4), le = da.number("linear_end", 2e-2);
  if (T < 1) FAIL(SDDM_ERR_INVALID_ARG, "n_timestep %d", T);
  std::vector<float> tabs((size_t)14 * (T + 1));
  if (compute_schedule(sched, T, ls, le, tabs.data())) FAIL(SDDM_ERR_NOT_IMPLEMENTED, "schedule '%s' (diffusion.py:84)", sched.c_str());
  c->net_type = net.string("type", "");
  if (c->net_type.empty()) {  // diffusion-only context: transitions / initial state
    c->T = T;
    c->tables.swap(tabs);
    c->tables_dirty = true;
    c->params.clear();
    c->plan_B = -1;
    c->lanes.clear();
    c->warena.reset();
    c->configured = true;
    return SDDM_OK;
  }
  if (c->net_type == "DiffWave") {                               // diffwave.py:113-131
    if (c->arch_type != "SDDM_spectrogram") FAIL(SDDM_ERR_NOT_IMPLEMENTED, "DiffWave needs arch SDDM_spectrogram");
    const Json& na = net.at("args");
    auto d = std::make_shared<DWState>();
    d->C = (int)na.number("residual_channels", 64);
    d->L = (int)na.number("residual_layers", 30);
    d->cycle = (int)na.number("dilation_cycle_length", 10);
    d->bins = (int)na.number("freq_bins", na.number("stft_bins", na.number("n_mels", 513)));
    d->hop = c->hop_samples;
    d->Kp = (d->bins + 31) / 32 * 32;
    if (d->C != 64) FAIL(SDDM_ERR_NOT_IMPLEMENTED, "DiffWave residual_channels %d (kernels are built for 64)", d->C);
    if (d->L < 1 || d->cycle < 1 || d->bins < 1) FAIL(SDDM_ERR_INVALID_ARG, "DiffWave geometry");
    if (d->hop != 256) FAIL(SDDM_ERR_NOT_IMPLEMENTED, "hop_samples %d: SpectrogramUpsampler upsamples x256", d->hop);
    c->T = T;
    c->tables.swap(tabs);
    c->tables_dirty = true;
    c->num_samples = -1;
    c->params.clear();
    for (const auto& kv : dw_param_shapes(*d)) {
      Param p;
      p.shape = kv.second;
      c->params[kv.first] = p;
    }
    c->params["diffusion_embedding.embedding_vector"].loaded = true;   // optional (default computed)
    c->dws = d;
    c->wgs.reset();
    c->params_dirty = true;
    c->plan_B = -1;
    c->lanes.clear();
    c->warena.reset();
    c->configured = true;
    return SDDM_OK;
  }
  if (c->net_type == "WaveGrad") {                               // wavegrad.py:140-179
    if (c->arch_type != "SDDM_spectrogram") FAIL(SDDM_ERR_NOT_IMPLEMENTED, "WaveGrad needs arch SDDM_spectrogram");
    if (c->hop_samples != WGState::kHop)
      FAIL(SDDM_ERR_NOT_IMPLEMENTED, "hop_samples %d: WaveGrad upsamples x300 (config_wavegrad.json:8)", c->hop_samples);
    c->T = T;
    c->tables.swap(tabs);
    c->tables_dirty = true;
    c->num_samples = -1;
    c->params.clear();
    for (const auto& kv : wg_param_shapes()) {
      Param p;
      p.shape = kv.second;
      c->params[kv.first] = p;
    }
    c->dws.reset();
    c->wgs = std::make_shared<WGState>();
    c->params_dirty = true;
    c->plan_B = -1;
    c->lanes.clear();
    c->warena.reset();
    c->configured = true;
    return SDDM_OK;
  }
  if (c->net_type != "UNetModified2") FAIL(SDDM_ERR_NOT_IMPLEMENTED, "network type '%s'", c->net_type.c_str());
  if (c->arch_type != "SDDM") FAIL(SDDM_ERR_NOT_IMPLEMENTED, "UNetModified2 under arch '%s'", c->arch_type.c_str());
  c->dws.reset();
  c->wgs.reset();
  const Json& na = net.at("args");
  UNetCfg u;
  u.in_channel = (int)na.number("in_channel", 2);
  u.out_channel = (int)na.number("out_channel", 1);
  u.inner = (int)na.number("inner_channel", 32);
  u.groups = (int)na.number("norm_groups", 32);
  u.mults = na.ints("channel_mults", {1, 2, 3, 4, 5});
  u.res_blocks = (int)na.number("res_blocks", 3);
  u.dropout = na.number("dropout", 0.0);
  u.seg = (int)na.number("segment_len", 128);
  u.stride = (int)na.number("segment_stride", 64);
  const int Ns = (int)cfg.number("num_samples", (double)na.number("num_samples", -1));
  if (u.in_channel != 2 || u.out_channel != 1)
    FAIL(SDDM_ERR_NOT_IMPLEMENTED, "UNetModified2 with in_channel %d / out_channel %d", u.in_channel, u.out_channel);
  if (u.inner > 128 || u.inner % 32) FAIL(SDDM_ERR_NOT_IMPLEMENTED, "inner_channel %d (multiples of 32 up to 128)", u.inner);
  if (Ns <= u.seg || (Ns - u.seg) % u.stride) FAIL(SDDM_ERR_SHAPE, "num_samples %d: (n - %d) %% %d != 0 (UNetModified2.py:13)", Ns, u.seg, u.stride);
  const int F = (Ns - u.seg) / u.stride + 1;
  const int div = 1 << (int)u.mults.size();
  if (F % div || u.seg % div) FAIL(SDDM_ERR_SHAPE, "n_frames %d and segment_len %d must be multiples of %d", F, u.seg, div);
  if (u.seg % u.stride) FAIL(SDDM_ERR_NOT_IMPLEMENTED, "segment_len %% segment_stride != 0");
  c->T = T;
  c->tables.swap(tabs);
  c->tables_dirty = true;
  c->ucfg = u;
  c->num_samples = Ns;
  c->params.clear();
  for (const auto& kv : unet_param_shapes(u)) {
    Param p;
    p.shape = kv.second;
    c->params[kv.first] = p;
  }
  c->params_dirty = true;
  c->plan_B = -1;
  c->lanes.clear();
  c->warena.reset();
  c->configured = true;
  return SDDM_OK;
}

int sddm_load_param(sddm_ctx* c, const char* key_c, const void* host_ptr, const int64_t* shape, int ndim,
                    int src_dtype) {
  if (!c || !c->configured) FAIL(SDDM_ERR_STATE, "context not configured");
  if (!key_c || !host_ptr || (ndim > 0 && !shape)) FAIL(SDDM_ERR_INVALID_ARG, "NULL argument");
  std::string key = key_c;
  if (key.rfind("module.", 0) == 0) key = key.substr(7);
  int64_t n = 1;
  for (int i = 0; i < ndim; ++i) n *= shape[i];
  auto read = [&](std::vector<float>& dst) -> int {
    dst.resize((size_t)n);
    if (src_dtype == DT_F32) std::memcpy(dst.data(), host_ptr, sizeof(float) * n);
    else if (src_dtype == DT_BF16) {
      for (int64_t i = 0; i < n; ++i) {
        uint32_t u = (uint32_t)((const uint16_t*)host_ptr)[i] << 16;
        std::memcpy(&dst[i], &u, 4);
      }
    } else if (src_dtype == DT_F16) {
      for (int64_t i = 0; i < n; ++i) dst[i] = (float)((const _Float16*)host_ptr)[i];
    } else {
      return 1;
    }
    return 0;
  };
  if (key.rfind("diffusion.", 0) == 0) {
    const std::string name = key.substr(10);
    for (int k = 0; k < 14; ++k)
      if (name == kTableNames[k]) {
        if (ndim != 1 || shape[0] != c->T + 1)
          FAIL(SDDM_ERR_SHAPE, "%s: expected [%d]", key.c_str(), c->T + 1);
        std::vector<float> v;
        if (read(v)) FAIL(SDDM_ERR_INVALID_ARG, "bad src dtype %d", src_dtype);
        std::memcpy(c->tables.data() + (size_t)k * (c->T + 1), v.data(), sizeof(float) * v.size());
        c->tables_dirty = true;
        return SDDM_OK;
      }
    FAIL(SDDM_ERR_INVALID_ARG, "unexpected key %s", key.c_str());
  }
  if (key.rfind("noise_estimate_model.", 0) == 0) key = key.substr(21);
  auto it = c->params.find(key);
  if (it == c->params.end()) FAIL(SDDM_ERR_INVALID_ARG, "unexpected key %s", key_c);
  Param& p = it->second;
  if ((int)p.shape.size() != ndim) FAIL(SDDM_ERR_SHAPE, "%s: rank %d != %d", key_c, ndim, (int)p.shape.size());
  for (int i = 0; i < ndim; ++i)
    if (p.shape[i] != shape[i]) FAIL(SDDM_ERR_SHAPE, "%s: shape mismatch in dim %d", key_c, i);
  if (read(p.data)) FAIL(SDDM_ERR_INVALID_ARG, "bad src dtype %d", src_dtype);
  p.loaded = true;
  c->params_dirty = true;
  return SDDM_OK;
}

int sddm_missing_params(sddm_ctx* c, int64_t* n_missing) {
  if (!c || !n_missing) FAIL(SDDM_ERR_INVALID_ARG, "NULL argument");
  int64_t m = 0;
  for (const auto& kv : c->params) m += kv.second.loaded ? 0 : 1;
  *n_missing = m;
  return SDDM_OK;
}

static int prepare_plan(sddm_ctx* c, int64_t B, int64_t N) {
  if (N != c->num_samples)
    FAIL(SDDM_ERR_SHAPE, "condition has %lld samples, network built for num_samples=%d", (long long)N, c->num_samples);
  if (B < 1 || B > 65535) FAIL(SDDM_ERR_INVALID_ARG, "batch %lld", (long long)B);
  if (c->plan_B != (int)B) return build_plan(c, (int)B);
  return SDDM_OK;
}

static int sample_impl(sddm_ctx* c, const float* cond, int64_t B, int64_t N, uint64_t seed, int64_t row_offset,
                       float* out, float* record, int sample_inter, void* stream, const float* noise = nullptr);

int sddm_sample(sddm_ctx* c, const float* cond, int64_t B, int64_t N, uint64_t seed, int64_t row_offset,
                float* out, void* stream) {
  return sample_impl(c, cond, B, N, seed, row_offset, out, nullptr, 0, stream);
}

int sddm_sample_noise(sddm_ctx* c, const float* cond, int64_t B, int64_t N, const float* noise, float* out,
                      void* stream) {
  if (!noise) FAIL(SDDM_ERR_INVALID_ARG, "NULL noise");
  return sample_impl(c, cond, B, N, 0, 0, out, nullptr, 0, stream, noise);
}

int sddm_sample_continuous(sddm_ctx* c, const float* cond, int64_t B, int64_t N, uint64_t seed,
                           int64_t row_offset, float* out, float* record, int sample_inter, void* stream) {
  if (!record || sample_inter < 1) FAIL(SDDM_ERR_INVALID_ARG, "record buffer / sample_inter");
  return sample_impl(c, cond, B, N, seed, row_offset, out, record, sample_inter, stream);
}

static int sample_impl(sddm_ctx* c, const float* cond, int64_t B, int64_t N, uint64_t seed, int64_t row_offset,
                       float* out, float* record, int sample_inter, void* stream, const float* noise) {
  int r = ensure_ready(c);
  if (r) return r;
  if (!cond || !out) FAIL(SDDM_ERR_INVALID_ARG, "NULL tensor");
  if (c->dws) return dw_sample(c, cond, B, N, seed, row_offset, out, record, sample_inter, noise, (hipStream_t)stream);
  if (c->wgs) return wg_sample(c, cond, B, N, seed, row_offset, out, record, sample_inter, noise, (hipStream_t)stream);
  r = prepare_plan(c, B, N);
  if (r) return r;
  hipStream_t user = (hipStream_t)stream;
  // (caller-supplied noise: the step graphs would bake its pointer; the per-launch path reads it)
  const bool graph = c->use_graphs && !c->prof && !record && !noise;
  const int T = c->T;
  StepParams* sp0 = c->warena.at<StepParams>(c->off_tdev);
  float* temb_tab = c->warena.at<float>(c->off_temb_tab);
  // noise-level embeddings of every t (same for all rows: model.py:108)
  EmbedArgs e{};
  e.table = c->dtab(3); e.time_step_mode = c->noise_time_step; e.R = T + 1; e.dim = c->ucfg.inner;
  e.emb_vec = c->warena.at<float>(c->woff.at("emb_vec"));
  e.w1 = c->warena.at<float>(c->woff.at("mlp.w1")); e.b1 = c->warena.at<float>(c->woff.at("mlp.b1"));
  e.w2 = c->warena.at<float>(c->woff.at("mlp.w2")); e.b2 = c->warena.at<float>(c->woff.at("mlp.b2"));
  e.pw = c->warena.at<float>(c->woff.at("proj.w")); e.pb = c->warena.at<float>(c->woff.at("proj.b"));
  e.SC = c->SC; e.out = temb_tab;
  SDDM_HIP_CHECK(launch_embed(e, user));
  // per-lane state: x_t (graph-stable copy when replaying graphs), condition rows, step counter
  for (auto& Lp : c->lanes) {
    Lane& L = *Lp;
    const int64_t rows = L.B, off = (int64_t)L.row0 * N;
    float* xb = graph ? L.arena.at<float>(L.off_x) : out + off;
    const float* cb = cond + off;
    if (graph) {
      SDDM_HIP_CHECK(hipMemcpyAsync(L.arena.at<float>(L.off_cond), cb, sizeof(float) * rows * N,
                                    hipMemcpyDeviceToDevice, user));
      cb = L.arena.at<float>(L.off_cond);
    }
    StepParams* sp = (StepParams*)((char*)sp0 + 64 * L.idx);
    InitArgs ia{};
    ia.mode = c->init_mode; ia.cond = cb; ia.out = xb; ia.total = rows * N; ia.N = N; ia.T = T;
    ia.co = c->coef(); ia.seed = seed; ia.row_offset = row_offset + L.row0;
    ia.noise = noise ? noise + off : nullptr;
    SDDM_HIP_CHECK(launch_init_state(ia, user));
    SDDM_HIP_CHECK(launch_set_params(sp, T + 1, seed, row_offset + L.row0, user));
    L.rs.cond = cb; L.rs.x = xb; L.rs.temb = temb_tab; L.rs.temb_per_b = 0; L.rs.t_dev = &sp->t;
    L.rs.final_mode = c->tr_mode; L.rs.eps_out = nullptr; L.rs.seed = seed; L.rs.row_offset = row_offset + L.row0;
    L.rs.noise = noise ? noise + off : nullptr; L.rs.noise_ld = B * N;
  }
  if (graph) {
    const int ns = std::min<int>(kStreams, (int)c->lanes.size());
    if (!c->ev_in) SDDM_HIP_CHECK(hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming));
    for (int k = 0; k < ns; ++k)
      if (!c->work[k]) {
        SDDM_HIP_CHECK(hipStreamCreateWithFlags(&c->work[k], hipStreamNonBlocking));
        SDDM_HIP_CHECK(hipEventCreateWithFlags(&c->ev_done[k], hipEventDisableTiming));
      }
    SDDM_HIP_CHECK(hipEventRecord(c->ev_in, user));
    for (int k = 0; k < ns; ++k) SDDM_HIP_CHECK(hipStreamWaitEvent(c->work[k], c->ev_in, 0));
    int K = 1;
    for (int k : {10, 8, 5, 4, 2})
      if (T % k == 0) { K = k; break; }
    for (auto& Lp : c->lanes) {   // capture K steps of every lane once per plan
      Lane& L = *Lp;
      if (L.gexec && L.g_gen == c->plan_gen && L.g_K == K) continue;
      if (L.gexec) { (void)hipGraphExecDestroy(L.gexec); L.gexec = nullptr; }
      if (L.graph) { (void)hipGraphDestroy(L.graph); L.graph = nullptr; }
      hipStream_t s = c->work[L.idx % ns];
      SDDM_HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int k = 0; k < K; ++k) {
        r = run_ops(c, L, s);
        if (r) {
          hipGraph_t junk = nullptr;
          (void)hipStreamEndCapture(s, &junk);
          if (junk) (void)hipGraphDestroy(junk);
          return r;
        }
      }
      SDDM_HIP_CHECK(hipStreamEndCapture(s, &L.graph));
      SDDM_HIP_CHECK(hipGraphInstantiate(&L.gexec, L.graph, nullptr, nullptr, 0));
      L.g_gen = c->plan_gen;
      L.g_K = K;
    }
    // lanes on different streams start with a phase offset (SDDM_LANE_OFFSET_US per lane index):
    // one lane's latency-bound deep levels then overlap another lane's bandwidth-bound wide levels
    static const int off_us = std::getenv("SDDM_LANE_OFFSET_US") ? std::atoi(std::getenv("SDDM_LANE_OFFSET_US")) : 0;
    if (off_us > 0)
      for (auto& Lp : c->lanes)
        if (Lp->idx % ns) SDDM_HIP_CHECK(launch_delay((unsigned)(off_us * (Lp->idx % ns)), c->work[Lp->idx % ns]));
    for (int i = 0; i < T / K; ++i)
      for (auto& Lp : c->lanes) SDDM_HIP_CHECK(hipGraphLaunch(Lp->gexec, c->work[Lp->idx % ns]));
    for (auto& Lp : c->lanes)
      SDDM_HIP_CHECK(hipMemcpyAsync(out + (int64_t)Lp->row0 * N, Lp->rs.x, sizeof(float) * Lp->B * N,
                                    hipMemcpyDeviceToDevice, c->work[Lp->idx % ns]));
    for (int k = 0; k < ns; ++k) {
      SDDM_HIP_CHECK(hipEventRecord(c->ev_done[k], c->work[k]));
      SDDM_HIP_CHECK(hipStreamWaitEvent(user, c->ev_done[k], 0));
    }
    return SDDM_OK;
  }
  int64_t nrec = 0;
  for (int t = T; t >= 1; --t) {
    for (auto& Lp : c->lanes) {
      r = run_ops(c, *Lp, user);
      if (r) return r;
    }
    if (record && t % sample_inter == 0) {  // model.py:100-101: keep x_{t-1} when t % inter == 0
      SDDM_HIP_CHECK(hipMemcpyAsync(record + nrec * B * N, out, sizeof(float) * B * N, hipMemcpyDeviceToDevice, user));
      ++nrec;
    }
  }
  return SDDM_OK;
}

int sddm_network_forward(sddm_ctx* c, const float* cond, const float* x_t, const float* noise_level, int64_t B,
                         int64_t N, float* eps_out, void* stream) {
  int r = ensure_ready(c);
  if (r) return r;
  if (!cond || !x_t || !noise_level || !eps_out) FAIL(SDDM_ERR_INVALID_ARG, "NULL tensor");
  if (c->dws) return dw_forward(c, cond, x_t, noise_level, B, N, eps_out, (hipStream_t)stream);
  if (c->wgs) return wg_forward(c, cond, x_t, noise_level, B, N, eps_out, (hipStream_t)stream);
  r = prepare_plan(c, B, N);
  if (r) return r;
  hipStream_t s = (hipStream_t)stream;
  for (auto& Lp : c->lanes) {
    Lane& L = *Lp;
    const int64_t off = (int64_t)L.row0 * N;
    float* temb = L.arena.at<float>(L.off_temb_fwd);
    EmbedArgs e{};
    e.noise_levels = noise_level + L.row0; e.R = L.B; e.dim = c->ucfg.inner;
    e.emb_vec = c->warena.at<float>(c->woff.at("emb_vec"));
    e.w1 = c->warena.at<float>(c->woff.at("mlp.w1")); e.b1 = c->warena.at<float>(c->woff.at("mlp.b1"));
    e.w2 = c->warena.at<float>(c->woff.at("mlp.w2")); e.b2 = c->warena.at<float>(c->woff.at("mlp.b2"));
    e.pw = c->warena.at<float>(c->woff.at("proj.w")); e.pb = c->warena.at<float>(c->woff.at("proj.b"));
    e.SC = c->SC; e.out = temb;
    SDDM_HIP_CHECK(launch_embed(e, s));
    L.rs.cond = cond + off; L.rs.x = const_cast<float*>(x_t) + off; L.rs.temb = temb; L.rs.temb_per_b = 1;
    L.rs.t_dev = nullptr; L.rs.final_mode = -1; L.rs.eps_out = eps_out + off; L.rs.seed = 0; L.rs.row_offset = 0;
    L.rs.noise = nullptr;
    r = run_ops(c, L, s);
    if (r) return r;
  }
  return SDDM_OK;
}

int sddm_transition(sddm_ctx* c, int mode, const float* x_t, const float* eps, const float* cond, int t, int64_t B,
                    int64_t N, uint64_t seed, int64_t row_offset, float* out, void* stream) {
  if (!c || !c->configured) FAIL(SDDM_ERR_STATE, "context not configured");
  if (mode < 0 || mode > 4) FAIL(SDDM_ERR_NOT_IMPLEMENTED, "transition mode %d", mode);
  if (t < 1 || t > c->T) FAIL(SDDM_ERR_INVALID_ARG, "t=%d outside [1, %d]", t, c->T);
  if (!x_t || !eps || !out || (mode >= 2 && mode <= 3 && !cond)) FAIL(SDDM_ERR_INVALID_ARG, "NULL tensor");
  SDDM_HIP_CHECK(hipSetDevice(c->device));
  if (!c->warena.base) {  // tables only (no network needed for a transition)
    c->warena.reset();
    c->off_tables = c->warena.reserve(sizeof(float) * 14 * (c->T + 1));
    c->off_tdev = c->warena.reserve(64 * kMaxLanes);
    SDDM_HIP_CHECK(c->warena.commit());
    c->params_dirty = true;
    c->tables_dirty = true;
  }
  if (c->tables_dirty) {
    const int r = upload_tables(c);
    if (r) return r;
  }
  TransArgs a{};
  a.mode = mode; a.x_t = x_t; a.eps = eps; a.cond = cond; a.out = out; a.total = B * N; a.N = N; a.t = t;
  a.co = c->coef(); a.seed = seed; a.row_offset = row_offset;
  SDDM_HIP_CHECK(launch_transition(a, (hipStream_t)stream));
  return SDDM_OK;
}

int sddm_q_sample(sddm_ctx* c, int mode, const float* x0, const float* y, const float* noise, const int64_t* t,
                  const float* r, int64_t B, int64_t N, float* x_t, float* combined, float* s_out, float* level_out,
                  void* stream) {
  if (!c || !c->configured) FAIL(SDDM_ERR_STATE, "context not configured");
  if (mode < 0 || mode > 1) FAIL(SDDM_ERR_NOT_IMPLEMENTED, "q_sample mode %d", mode);
  if (!x0 || !noise || !t || !x_t || (mode == 1 && !y)) FAIL(SDDM_ERR_INVALID_ARG, "NULL tensor");
  if (B < 0 || N < 1) FAIL(SDDM_ERR_INVALID_ARG, "shape B=%lld N=%lld", (long long)B, (long long)N);
  SDDM_HIP_CHECK(hipSetDevice(c->device));
  if (!c->warena.base) {  // tables only
    c->warena.reset();
    c->off_tables = c->warena.reserve(sizeof(float) * 14 * (c->T + 1));
    c->off_tdev = c->warena.reserve(64 * kMaxLanes);
    SDDM_HIP_CHECK(c->warena.commit());
    c->params_dirty = true;
    c->tables_dirty = true;
  }
  if (c->tables_dirty) {
    const int rr = upload_tables(c);
    if (rr) return rr;
  }
  QArgs a{};
  a.mode = mode; a.x0 = x0; a.y = y; a.noise = noise; a.t = t; a.r = r;
  a.sab = c->dtab(3); a.alpha_bar = c->dtab(2); a.m = c->dtab(8); a.sqrt_delta = c->dtab(9);
  a.x_t = x_t; a.combined = combined; a.s_out = s_out; a.level_out = level_out; a.B = B; a.N = N;
  SDDM_HIP_CHECK(launch_q_sample(a, (hipStream_t)stream));
  return SDDM_OK;
}

int sddm_set_conv_tuning(sddm_ctx* c, const char* json) {
  if (!c || !json) FAIL(SDDM_ERR_INVALID_ARG, "NULL argument");
  Json j;
  try {
    j = Json::parse(json);
  } catch (const std::exception& e) {
    FAIL(SDDM_ERR_INVALID_ARG, "tuning JSON: %s", e.what());
  }
  // one table, or {"tables": [table, ...]}: the plan takes the first whose lane batch, dtype and
  // length match it (a bf16 table also serves f16 plans)
  std::vector<const Json*> tabs;
  if (j.has("tables")) {
    const Json& arr = j.at("tables");
    if (arr.kind != Json::ARR) FAIL(SDDM_ERR_INVALID_ARG, "tables: a list");
    for (const auto& t : arr.arr) tabs.push_back(&t);
  } else {
    tabs.push_back(&j);
  }
  std::vector<sddm_ctx::TuneTable> out;
  for (const Json* tp : tabs) {
    const Json& t = *tp;
    if (t.kind != Json::OBJ) FAIL(SDDM_ERR_INVALID_ARG, "tuning table: an object");
    sddm_ctx::TuneTable tt;
    const std::string dts = t.string("dtype", "");
    tt.dtype = dts == "float32" ? DT_F32 : dts == "bfloat16" ? DT_BF16 : dts == "float16" ? DT_F16 : -1;
    if (t.has("deep"))
      for (const auto& kv : t.at("deep").obj) {
        if (kv.second.kind != Json::ARR || kv.second.arr.size() != 2) FAIL(SDDM_ERR_INVALID_ARG, "deep.%s: [mt, nw]", kv.first.c_str());
        tt.deep_tune[kv.first] = {(int)kv.second.arr[0].num, (int)kv.second.arr[1].num};
      }
    // "kernel": {"<layer>": "strip" | "tile:<cfg>" | "deep" | "deep:<mt>:<nw>[:<nb>]" | "chain"}
    if (t.has("kernel"))
      for (const auto& kv : t.at("kernel").obj) {
        if (kv.second.kind != Json::STR) FAIL(SDDM_ERR_INVALID_ARG, "kernel.%s: a string", kv.first.c_str());
        const std::string& v = kv.second.str;
        sddm_ctx::KernTune k{0, 0, 0, 0};
        if (v == "strip") k.kind = 1;
        else if (v.rfind("tile:", 0) == 0) { k.kind = 2; k.a = std::atoi(v.c_str() + 5); }
        else if (v == "deep") k.kind = 3;
        else if (v.rfind("deep:", 0) == 0) { k.kind = 3; std::sscanf(v.c_str() + 5, "%d:%d:%d", &k.a, &k.b, &k.c); }
        else if (v == "chain") k.kind = 4;
        else FAIL(SDDM_ERR_INVALID_ARG, "kernel.%s: unknown choice '%s'", kv.first.c_str(), v.c_str());
        if (k.kind == 2 && (k.a < 0 || k.a >= conv_tile_ncfg())) FAIL(SDDM_ERR_INVALID_ARG, "kernel.%s: tile configuration %d", kv.first.c_str(), k.a);
        tt.kern_tune[kv.first] = k;
      }
    tt.B = (int)t.number("lane_batch", -1);
    tt.N = (int)t.number("num_samples", -1);
    out.push_back(std::move(tt));
  }
  c->tunes = std::move(out);
  c->plan_B = -1;                                   // re-plan on the next call
  c->lanes.clear();
  return SDDM_OK;
}

int sddm_log_spectrogram(const float* audio, int64_t B, int64_t N, int n_fft, int hop, const float* window,
                         const float* fb, int n_out, float* out, void* stream) {
  if (!audio || !window || !out) FAIL(SDDM_ERR_INVALID_ARG, "NULL tensor");
  if (n_fft < 2 || n_fft > 1024 || (n_fft & (n_fft - 1))) FAIL(SDDM_ERR_NOT_IMPLEMENTED, "n_fft %d (powers of two <= 1024)", n_fft);
  if (hop < 1 || B < 1 || N <= n_fft / 2) FAIL(SDDM_ERR_SHAPE, "B=%lld N=%lld hop=%d n_fft=%d", (long long)B, (long long)N, hop, n_fft);
  if (!fb && n_out != n_fft / 2 + 1) FAIL(SDDM_ERR_INVALID_ARG, "linear spectrogram has %d bins, not %d", n_fft / 2 + 1, n_out);
  StftArgs a{};
  a.audio = audio; a.B = B; a.N = N; a.n_fft = n_fft; a.hop = hop; a.frames = (int)(1 + N / hop); a.n_out = n_out;
  a.window = window; a.fb = fb; a.out = out;
  SDDM_HIP_CHECK(launch_stft_features(a, (hipStream_t)stream));
  return SDDM_OK;
}

int sddm_initial_state(sddm_ctx* c, int mode, const float* cond, int64_t B, int64_t N, uint64_t seed,
                       int64_t row_offset, float* out, void* stream) {
  if (!c || !c->configured) FAIL(SDDM_ERR_STATE, "context not configured");
  if (mode < 0 || mode > 4) FAIL(SDDM_ERR_NOT_IMPLEMENTED, "init mode %d", mode);
  if (!out || (mode >= 2 && !cond)) FAIL(SDDM_ERR_INVALID_ARG, "NULL tensor");
  SDDM_HIP_CHECK(hipSetDevice(c->device));
  if (!c->warena.base) {
    c->warena.reset();
    c->off_tables = c->warena.reserve(sizeof(float) * 14 * (c->T + 1));
    c->off_tdev = c->warena.reserve(64 * kMaxLanes);
    SDDM_HIP_CHECK(c->warena.commit());
    c->params_dirty = true;
    c->tables_dirty = true;
  }
  if (c->tables_dirty) {
    const int r = upload_tables(c);
    if (r) return r;
  }
  InitArgs ia{};
  ia.mode = mode; ia.cond = cond; ia.out = out; ia.total = B * N; ia.N = N; ia.T = c->T;
  ia.co = c->coef(); ia.seed = seed; ia.row_offset = row_offset;
  SDDM_HIP_CHECK(launch_init_state(ia, (hipStream_t)stream));
  return SDDM_OK;
}

int sddm_profile_enable(sddm_ctx* c, int enable) {
  if (!c) FAIL(SDDM_ERR_INVALID_ARG, "NULL ctx");
  SDDM_HIP_CHECK(hipSetDevice(c->device));
  c->prof = enable != 0;
  c->ev_pend.clear();
  c->op_acc.clear();
  if (c->prof && c->ev_pool.empty()) {
    c->ev_pool.resize(512);
    for (auto& e : c->ev_pool) SDDM_HIP_CHECK(hipEventCreate(&e));
  }
  return SDDM_OK;
}

static const std::vector<Op>& profiled_ops(sddm_ctx* c) {
  static const std::vector<Op> kNoOps;
  return c->lanes.empty() ? kNoOps : c->lanes[0]->ops;   // the same layer list in every lane
}

int sddm_profile_read(sddm_ctx* c, const char* kernel_class, double* avg_ms, int64_t* launches,
                      double* bytes_per_launch, double* flops_per_launch) {
  if (!c || !kernel_class) FAIL(SDDM_ERR_INVALID_ARG, "NULL argument");
  const std::string k = kernel_class;
  const int cls = k == "conv_in" ? 0 : k == "gn_finalize" ? 1 : k == "conv3x3" ? 2 : k == "final" ? 3 : -1;
  if (cls < 0) FAIL(SDDM_ERR_INVALID_ARG, "kernel class %s", kernel_class);
  const std::vector<Op>& ops = profiled_ops(c);
  double ms = 0, bytes = 0, flops = 0;
  int64_t n = 0;
  for (size_t i = 0; i < c->op_acc.size() && i < ops.size(); ++i) {
    if (ops[i].cls != cls) continue;
    ms += c->op_acc[i].ms; bytes += c->op_acc[i].bytes; flops += c->op_acc[i].flops; n += c->op_acc[i].n;
  }
  if (avg_ms) *avg_ms = n ? ms / n : 0.0;
  if (launches) *launches = n;
  if (bytes_per_launch) *bytes_per_launch = n ? bytes / n : 0.0;
  if (flops_per_launch) *flops_per_launch = n ? flops / n : 0.0;
  return SDDM_OK;
}

// profiling builds only (not part of the C ABI): copy the phase stamps of the op named by the
// SDDM_STAMPS environment variable, [blocks][8] u64
int sddm_debug_stamps(sddm_ctx* c, void* host, int64_t max_blocks, int64_t* n_blocks) {
  if (!c || !host || !n_blocks) FAIL(SDDM_ERR_INVALID_ARG, "NULL argument");
  *n_blocks = 0;
  if (!c->stamp_buf) return SDDM_OK;
  const int64_t n = std::min<int64_t>(c->stamp_blocks, max_blocks);
  SDDM_HIP_CHECK(hipDeviceSynchronize());
  SDDM_HIP_CHECK(hipMemcpy(host, c->stamp_buf, sizeof(unsigned long long) * 8 * n, hipMemcpyDeviceToHost));
  *n_blocks = n;
  return SDDM_OK;
}

int sddm_profile_ops(sddm_ctx* c, char* buf, int64_t buflen) {
  if (!c || !buf || buflen < 3) FAIL(SDDM_ERR_INVALID_ARG, "NULL argument");
  const std::vector<Op>& ops = profiled_ops(c);
  std::string js = "[";
  char tmp[768];
  for (size_t i = 0; i < ops.size(); ++i) {
    const ProfAcc a = i < c->op_acc.size() ? c->op_acc[i] : ProfAcc{};
    snprintf(tmp, sizeof(tmp),
             "%s{\"name\": \"%s\", \"kernel\": \"%s\", \"inst\": \"%s\", \"cls\": %d, \"launches\": %lld, "
             "\"avg_ms\": %.6f, \"bytes\": %.0f, \"flops\": %.0f}",
             i ? ", " : "", ops[i].name.c_str(), ops[i].kname.c_str(), ops[i].kinst.c_str(), ops[i].cls, (long long)a.n,
             a.n ? a.ms / a.n : 0.0, ops[i].bytes, ops[i].flops);
    js += tmp;
  }
  js += "]";
  if ((int64_t)js.size() + 1 > buflen) FAIL(SDDM_ERR_INVALID_ARG, "buffer too small (%zu)", js.size() + 1);
  std::memcpy(buf, js.c_str(), js.size() + 1);
  return SDDM_OK;
}

}  // extern "C"
