// WaveGrad path of the runtime (included by sddm_runtime.cpp after sddm_ctx): configuration,
// weight packing, workspace and the SDDM_spectrogram.infer loop (reference model/model.py:212-257,
// model/wavegrad.py).  Kernels: wavegrad.hip.
//
// The reference wiring of SDDM_spectrogram + WaveGrad fails (x_t [B,1,N] reaches a
// Conv1d as 4-D, and the squeezed [B,N] output broadcasts against x_t); the library applies the
// adapter: audio = x_t[:, 0], noise level [B], eps -> [B,1,N].
//
// Step-invariant per sampling call (the spectrogram does not change across steps): the spectrogram
// transpose, first_conv, and upsample.0's block1 and block2[0] (no FiLM reaches them).  The
// PositionalEncoding rows of all t are one launch.  Per reverse step: downsample.0, 5 FiLMs
// (2 convs each), 4 DBlocks (4 convs), upsample.0 (3 convs), upsample.1-4 (5 convs), last_conv,
// transition -- 52 launches.
#pragma once
#include "wg_kernels.h"

struct WGState {
  static constexpr int kHop = 300;                    // 5 * 5 * 3 * 2 * 2
  static constexpr int kSpecC = 128;
  static constexpr int kEncN = 1056;                  // 32 + 128 + 128 + 256 + 512
  std::map<std::string, size_t> woff;                 // packed weights in ctx->warena
  size_t off_tables = 0, off_sp = 0, off_enctab = 0, off_ev = 0;
  Arena act;                                          // activations of the current (B, F)
  std::map<std::string, size_t> aoff;
  int B = -1, F = -1;
};

namespace wg {
struct Down { int ci, co, f; };
struct Film { int ci, co; };
struct Up { int ci, h, f; int dil[4]; };
static const Down kDown[5] = {{1, 32, 1}, {32, 128, 2}, {128, 128, 2}, {128, 256, 3}, {256, 512, 5}};  // wavegrad.py:143-149
static const Film kFilm[5] = {{32, 128}, {128, 128}, {128, 256}, {256, 512}, {512, 512}};           // wavegrad.py:150-156
static const Up kUp[5] = {{768, 512, 5, {1, 2, 1, 2}}, {512, 512, 5, {1, 2, 1, 2}}, {512, 256, 3, {1, 2, 4, 8}},
                          {256, 128, 2, {1, 2, 4, 8}}, {128, 128, 2, {1, 2, 4, 8}}};                  // wavegrad.py:157-163
static const int kEncOff[5] = {0, 32, 160, 288, 544};
}  // namespace wg

// state-dict shapes of WaveGrad (wavegrad.py:140-165) without the noise_estimate_model. prefix
static std::map<std::string, std::vector<int64_t>> wg_param_shapes() {
  std::map<std::string, std::vector<int64_t>> s;
  auto conv = [&](const std::string& p, int co, int ci, int k) {
    s[p + ".weight"] = {co, ci, k};
    s[p + ".bias"] = {co};
  };
  conv("downsample.0", 32, 1, 5);
  for (int i = 1; i < 5; ++i) {
    const wg::Down& d = wg::kDown[i];
    const std::string p = "downsample." + std::to_string(i) + ".";
    conv(p + "residual_dense", d.co, d.ci, 1);
    conv(p + "conv.0", d.co, d.ci, 3);
    conv(p + "conv.1", d.co, d.co, 3);
    conv(p + "conv.2", d.co, d.co, 3);
  }
  for (int i = 0; i < 5; ++i) {
    const std::string p = "film." + std::to_string(i) + ".";
    conv(p + "input_conv", wg::kFilm[i].ci, wg::kFilm[i].ci, 3);
    conv(p + "output_conv", 2 * wg::kFilm[i].co, wg::kFilm[i].ci, 3);
  }
  for (int i = 0; i < 5; ++i) {
    const wg::Up& u = wg::kUp[i];
    const std::string p = "upsample." + std::to_string(i) + ".";
    conv(p + "block1", u.h, u.ci, 1);
    conv(p + "block2.0", u.h, u.ci, 3);
    conv(p + "block2.1", u.h, u.h, 3);
    conv(p + "block3.0", u.h, u.h, 3);
    conv(p + "block3.1", u.h, u.h, 3);
  }
  conv("first_conv", 768, 128, 3);
  conv("last_conv", 1, 128, 3);
  return s;
}

static int wg_upload_weights(sddm_ctx* c) {
  WGState& d = *c->wgs;
  const int dt = c->dtype;
  const size_t es = dtype_size(dt);
  c->warena.reset();
  d.woff.clear();
  Arena& A = c->warena;
  struct Blob { size_t off; std::vector<char> bytes; };
  std::vector<Blob> blobs;
  auto add_f32 = [&](const std::string& name, const std::vector<float>& v) {
    Blob b;
    b.bytes.resize(v.size() * 4);
    std::memcpy(b.bytes.data(), v.data(), b.bytes.size());
    b.off = A.reserve(b.bytes.size());
    d.woff[name] = b.off;
    blobs.push_back(std::move(b));
  };
  // Conv1d weight [Cout][Cin][K] -> [Cout_pad64][K][Cin] in the compute dtype (zero pad rows)
  for (const auto& kv : wg_param_shapes()) {
    const std::string& key = kv.first;
    if (key.size() < 7 || key.compare(key.size() - 7, 7, ".weight")) continue;
    const std::string base = key.substr(0, key.size() - 7);
    const std::vector<float>& w = c->params.at(key).data;
    const int co = (int)kv.second[0], ci = (int)kv.second[1], k = (int)kv.second[2];
    add_f32(base + ".b", c->params.at(base + ".bias").data);
    if (base == "downsample.0") { add_f32(base + ".w", w); continue; }   // fp32 [32][1][5], VALU kernel
    const int cop = (co + 63) / 64 * 64;
    Blob b;
    b.bytes.assign((size_t)cop * k * ci * es, 0);
    for (int o = 0; o < co; ++o)
      for (int i = 0; i < ci; ++i)
        for (int t = 0; t < k; ++t) store_elem(b.bytes.data(), ((size_t)o * k + t) * ci + i, w[((size_t)o * ci + i) * k + t], dt);
    b.off = A.reserve(b.bytes.size());
    d.woff[base + ".w"] = b.off;
    blobs.push_back(std::move(b));
  }
  {  // PositionalEncoding exp vectors, torch fp32 op order (wavegrad.py:45-47)
    std::vector<float> ev;
    for (int i = 0; i < 5; ++i) {
      const int cnt = wg::kFilm[i].ci / 2;
      for (int k = 0; k < cnt; ++k) {
        const float step = (float)k / (float)cnt;
        ev.push_back(std::exp((float)(-std::log(1e4)) * step));
      }
    }
    add_f32("enc.ev", ev);
  }
  d.off_tables = A.reserve(sizeof(float) * 14 * (c->T + 1));
  d.off_sp = A.reserve(64);
  d.off_enctab = A.reserve(sizeof(float) * (size_t)(c->T + 1) * WGState::kEncN);
  c->off_tables = d.off_tables;
  SDDM_HIP_CHECK(A.commit());
  for (const auto& b : blobs) SDDM_HIP_CHECK(hipMemcpy(A.base + b.off, b.bytes.data(), b.bytes.size(), hipMemcpyHostToDevice));
  c->params_dirty = false;
  c->tables_dirty = true;
  d.B = -1;
  return SDDM_OK;
}

// activation buffers for (B, F): name -> [B][len][C] in the compute dtype
static int wg_prepare(sddm_ctx* c, int B, int F) {
  WGState& d = *c->wgs;
  if (d.B == B && d.F == F) return SDDM_OK;
  const size_t es = dtype_size(c->dtype);
  Arena& A = d.act;
  A.reset();
  d.aoff.clear();
  auto buf = [&](const std::string& n, int64_t len, int C) { d.aoff[n] = A.reserve(es * (size_t)B * len * C); };
  int64_t L[6];
  L[0] = (int64_t)WGState::kHop * F;
  for (int i = 1; i < 5; ++i) L[i] = L[i - 1] / wg::kDown[i].f;
  L[5] = F;
  buf("d0", L[0], 32);
  for (int i = 0; i < 5; ++i) {
    const std::string s = std::to_string(i);
    if (i > 0) for (const char* n : {"r", "a", "b", ""}) buf("d" + s + n, L[i], wg::kDown[i].co);
    buf("f" + s + "a", L[i], wg::kFilm[i].ci);
    buf("f" + s, L[i], 2 * wg::kFilm[i].co);
  }
  buf("spec", L[5], WGState::kSpecC);
  buf("uin", L[5], 768);
  for (int i = 0; i < 5; ++i) {
    const std::string s = std::to_string(i);
    const int64_t lin = L[5 - i], lout = L[4 - i];
    buf("u" + s + "b1", lin, wg::kUp[i].h);
    for (const char* n : {"y0", "x", "z", "", "m", "p"}) buf("u" + s + n, lout, wg::kUp[i].h);   // m: leaky(film(x)); p: pre-2 fallback scratch
  }
  d.aoff["eps"] = A.reserve(sizeof(float) * (size_t)B * L[0]);
  d.aoff["encb"] = A.reserve(sizeof(float) * (size_t)B * WGState::kEncN);
  SDDM_HIP_CHECK(A.commit());
  d.B = B;
  d.F = F;
  return SDDM_OK;
}

struct WGConvSpec {
  const char* src; int64_t src_T; int src_C; int map, f; int64_t Tc; int Cin;
  std::string w; int Cout, K, dil, pre; const char* film;
  int post, enc_off; const char* res; int res_map, res_f; int64_t res_T;
  const char* out;
  const char* efilm = nullptr; int post_film = 0; const char* out2 = nullptr;   // WGConvArgs::post_film
};

static int wg_conv(sddm_ctx* c, WGConvSpec q, int B, const float* enc, int enc_per_b, const int* t_dev,
                   hipStream_t s) {
  WGState& d = *c->wgs;
  const Arena& W = c->warena;
  std::string mod;
  WGConvArgs probe{};
  probe.Cout = q.Cout; probe.K = q.K; probe.dil = q.dil; probe.pre = q.pre; probe.out_f32 = 0;
  if (q.pre == 2 && !wg_conv_uses_lds(probe)) {   // modulate once into the UBlock's scratch, then a plain conv
    mod = std::string(q.out).substr(0, 2) + "p";
    WGFilmArgs fa{d.act.base + d.aoff.at(q.src), d.act.base + d.aoff.at(q.film), d.act.base + d.aoff.at(mod),
                  (int64_t)B * q.Tc, q.Cin};
    SDDM_HIP_CHECK(launch_wg_film(c->dtype, fa, s));
    q.src = mod.c_str();
    q.pre = 0;
    q.film = nullptr;
  }
  WGConvArgs a{};
  a.src = d.act.base + d.aoff.at(q.src); a.src_T = (int)q.src_T; a.src_C = q.src_C; a.map = q.map; a.f = q.f;
  a.Tc = (int)q.Tc; a.Cin = q.Cin; a.K = q.K; a.dil = q.dil; a.pre = q.pre;
  a.film = q.film ? d.act.base + d.aoff.at(q.film) : nullptr;
  a.w = W.base + d.woff.at(q.w + ".w"); a.bias = W.at<float>(d.woff.at(q.w + ".b")); a.Cout = q.Cout;
  a.post = q.post; a.enc = enc; a.enc_stride = WGState::kEncN; a.enc_off = q.enc_off; a.enc_per_b = enc_per_b;
  a.t_dev = t_dev;
  a.res = q.res ? d.act.base + d.aoff.at(q.res) : nullptr; a.res_map = q.res_map; a.res_f = q.res_f;
  a.res_T = (int)q.res_T;
  a.out = d.act.base + d.aoff.at(q.out); a.out_f32 = std::strcmp(q.out, "eps") == 0;
  a.B = B;
  a.post_film = q.post_film;
  a.efilm = q.efilm ? d.act.base + d.aoff.at(q.efilm) : nullptr;
  a.out2 = q.out2 ? d.act.base + d.aoff.at(q.out2) : nullptr;
  const hipError_t e = launch_wg_conv(c->dtype, a, s);
  if (e != hipSuccess) FAIL(SDDM_ERR_HIP, "wg_conv %s: %s", q.w.c_str(), hipGetErrorString(e));
  return SDDM_OK;
}

#define WG_TRY(x) do { const int _r = (x); if (_r) return _r; } while (0)

static void wg_lengths(int F, int64_t* L) {
  L[0] = (int64_t)WGState::kHop * F;
  for (int i = 1; i < 5; ++i) L[i] = L[i - 1] / wg::kDown[i].f;
  L[5] = F;
}

// step-invariant work of one call (wavegrad.py:175-177 for upsample.0's block1 / block2[0])
static int wg_condition(sddm_ctx* c, const float* spec, int B, int F, hipStream_t s) {
  WGState& d = *c->wgs;
  int64_t L[6];
  wg_lengths(F, L);
  WGSpecArgs sa{spec, d.act.base + d.aoff.at("spec"), B, WGState::kSpecC, F};
  SDDM_HIP_CHECK(launch_wg_spec(c->dtype, sa, s));
  WG_TRY(wg_conv(c, {"spec", L[5], 128, WG_MAP_ID, 1, L[5], 128, "first_conv", 768, 3, 1, 0, nullptr, 0, 0, nullptr, 0, 1, 0, "uin"},
                 B, nullptr, 0, nullptr, s));
  const wg::Up& u = wg::kUp[0];
  WG_TRY(wg_conv(c, {"uin", L[5], 768, WG_MAP_ID, 1, L[5], 768, "upsample.0.block1", u.h, 1, 1, 0, nullptr, 0, 0, nullptr, 0, 1, 0, "u0b1"},
                 B, nullptr, 0, nullptr, s));
  WG_TRY(wg_conv(c, {"uin", L[5], 768, WG_MAP_UP, u.f, L[4], 768, "upsample.0.block2.0", u.h, 3, u.dil[0], 1, nullptr, 0, 0,
                     nullptr, 0, 1, 0, "u0y0"}, B, nullptr, 0, nullptr, s));
  return SDDM_OK;
}

// one WaveGrad forward: audio [B][N] fp32 -> eps [B][N] fp32 (aoff "eps")
static int wg_network(sddm_ctx* c, const float* audio, int B, int F, const float* enc, int enc_per_b, int* t_dev,
                      hipStream_t s) {
  WGState& d = *c->wgs;
  const Arena& W = c->warena;
  int64_t L[6];
  wg_lengths(F, L);
  WGFirstArgs fa{audio, W.at<float>(d.woff.at("downsample.0.w")), W.at<float>(d.woff.at("downsample.0.b")),
                 d.act.base + d.aoff.at("d0"), B, (int)L[0], t_dev};
  SDDM_HIP_CHECK(launch_wg_first(c->dtype, fa, s));
  std::string x = "d0";
  for (int i = 0; i < 5; ++i) {
    const std::string si = std::to_string(i);
    if (i > 0) {                                         // DBlock (wavegrad.py:126-137)
      const wg::Down& dn = wg::kDown[i];
      const std::string p = "downsample." + si + ".", o = "d" + si;
      const char* xs = x.c_str();
      WG_TRY(wg_conv(c, {xs, L[i - 1], dn.ci, WG_MAP_DOWN, dn.f, L[i], dn.ci, p + "residual_dense", dn.co, 1, 1, 0, nullptr, 0, 0,
                         nullptr, 0, 1, 0, (o + "r").c_str()}, B, enc, enc_per_b, t_dev, s));
      WG_TRY(wg_conv(c, {xs, L[i - 1], dn.ci, WG_MAP_DOWN, dn.f, L[i], dn.ci, p + "conv.0", dn.co, 3, 1, 1, nullptr, 0, 0,
                         nullptr, 0, 1, 0, (o + "a").c_str()}, B, enc, enc_per_b, t_dev, s));
      WG_TRY(wg_conv(c, {(o + "a").c_str(), L[i], dn.co, WG_MAP_ID, 1, L[i], dn.co, p + "conv.1", dn.co, 3, 2, 1, nullptr, 0, 0,
                         nullptr, 0, 1, 0, (o + "b").c_str()}, B, enc, enc_per_b, t_dev, s));
      WG_TRY(wg_conv(c, {(o + "b").c_str(), L[i], dn.co, WG_MAP_ID, 1, L[i], dn.co, p + "conv.2", dn.co, 3, 4, 1, nullptr, 0, 0,
                         (o + "r").c_str(), WG_MAP_ID, 1, L[i], o.c_str()}, B, enc, enc_per_b, t_dev, s));
      x = o;
    }
    const wg::Film& fm = wg::kFilm[i];                   // FiLM (wavegrad.py:66-71)
    const std::string p = "film." + si + ".", o = "f" + si;
    WG_TRY(wg_conv(c, {x.c_str(), L[i], fm.ci, WG_MAP_ID, 1, L[i], fm.ci, p + "input_conv", fm.ci, 3, 1, 0, nullptr, 1,
                       wg::kEncOff[i], nullptr, 0, 1, 0, (o + "a").c_str()}, B, enc, enc_per_b, t_dev, s));
    WG_TRY(wg_conv(c, {(o + "a").c_str(), L[i], fm.ci, WG_MAP_ID, 1, L[i], fm.ci, p + "output_conv", 2 * fm.co, 3, 1, 0, nullptr,
                       0, 0, nullptr, 0, 1, 0, o.c_str()}, B, enc, enc_per_b, t_dev, s));
  }
  x = "uin";
  for (int i = 0; i < 5; ++i) {                           // UBlock (wavegrad.py:91-112)
    const wg::Up& u = wg::kUp[i];
    const std::string si = std::to_string(i), p = "upsample." + si + ".", o = "u" + si;
    const std::string film = "f" + std::to_string(4 - i);
    const int64_t lin = L[5 - i], lout = L[4 - i];
    // FiLM placement.  512-channel UBlocks (upsample.0-1): the FiLM of block2.1 / block3.0 /
    // block3.1's inputs runs in their producers' epilogues (post_film: y0 holds leaky(film(block2.0
    // out)), m holds leaky(film(x)), z holds leaky(film(block3.0 out))), so shift / scale are read
    // once per element instead of once per 128-channel block of the consumer (upsample.1: 1137 ->
    // 962 us per step at B=64).  upsample.0's block2.0 is step-invariant (wg_condition), so its
    // block2.1 keeps the FiLM in the staging (pre 2).  The 128 / 256-channel UBlocks keep the
    // staged FiLM: there the epilogue loads are exposed (all blocks reach their epilogues
    // together) and cost more than the re-reads save (upsample.4: 1324 -> 1675 us)
    const std::string ym = o + "y0", xm = o + "m", xo = o + "x", zo = o + "z", b1 = o + "b1";
    static const int epi_min_h = std::getenv("SDDM_WG_EPI_MIN_H") ? std::atoi(std::getenv("SDDM_WG_EPI_MIN_H")) : 512;
    const bool epi = u.h >= epi_min_h;
    if (i > 0) {
      WG_TRY(wg_conv(c, {x.c_str(), lin, u.ci, WG_MAP_ID, 1, lin, u.ci, p + "block1", u.h, 1, 1, 0, nullptr, 0, 0, nullptr, 0, 1, 0,
                         b1.c_str()}, B, enc, enc_per_b, t_dev, s));
      WG_TRY(wg_conv(c, {x.c_str(), lin, u.ci, WG_MAP_UP, u.f, lout, u.ci, p + "block2.0", u.h, 3, u.dil[0], 1, nullptr, 0, 0,
                         nullptr, 0, 1, 0, ym.c_str(), epi ? film.c_str() : nullptr, epi ? 1 : 0}, B, enc, enc_per_b, t_dev, s));
    }
    const bool pre21 = !epi || i == 0;
    WG_TRY(wg_conv(c, {ym.c_str(), lout, u.h, WG_MAP_ID, 1, lout, u.h, p + "block2.1", u.h, 3, u.dil[1], pre21 ? 2 : 0,
                       pre21 ? film.c_str() : nullptr, 0, 0, b1.c_str(), WG_MAP_UP, u.f, lin, xo.c_str(),
                       epi ? film.c_str() : nullptr, epi ? 2 : 0, epi ? xm.c_str() : nullptr}, B, enc, enc_per_b, t_dev, s));
    WG_TRY(wg_conv(c, {epi ? xm.c_str() : xo.c_str(), lout, u.h, WG_MAP_ID, 1, lout, u.h, p + "block3.0", u.h, 3, u.dil[2],
                       epi ? 0 : 2, epi ? nullptr : film.c_str(), 0, 0, nullptr, 0, 1, 0, zo.c_str(), epi ? film.c_str() : nullptr,
                       epi ? 1 : 0}, B, enc, enc_per_b, t_dev, s));
    WG_TRY(wg_conv(c, {zo.c_str(), lout, u.h, WG_MAP_ID, 1, lout, u.h, p + "block3.1", u.h, 3, u.dil[3], epi ? 0 : 2,
                       epi ? nullptr : film.c_str(), 0, 0, xo.c_str(), WG_MAP_ID, 1, lout, o.c_str()}, B, enc, enc_per_b, t_dev, s));
    x = o;
  }
  WG_TRY(wg_conv(c, {x.c_str(), L[0], 128, WG_MAP_ID, 1, L[0], 128, "last_conv", 1, 3, 1, 0, nullptr, 0, 0, nullptr, 0, 1, 0, "eps"},
                 B, enc, enc_per_b, t_dev, s));
  return SDDM_OK;
}

static int wg_enc(sddm_ctx* c, const float* noise_levels, int rows, float* out, hipStream_t s) {
  WGState& d = *c->wgs;
  WGEncArgs e{};
  e.noise_levels = noise_levels; e.table = c->warena.at<float>(d.off_tables) + (size_t)3 * (c->T + 1);
  e.time_step_mode = c->noise_time_step; e.R = rows;
  e.ev = c->warena.at<float>(d.woff.at("enc.ev")); e.stride = WGState::kEncN; e.n = WGState::kEncN;
  for (int i = 0; i < 5; ++i) { e.dims[i] = wg::kFilm[i].ci; e.offs[i] = wg::kEncOff[i]; }
  e.out = out;
  SDDM_HIP_CHECK(launch_wg_enc(e, s));
  return SDDM_OK;
}

static int wg_check_shape(sddm_ctx* c, int64_t B, int64_t N, int* F) {
  if (B < 1 || B > 65535) FAIL(SDDM_ERR_INVALID_ARG, "batch %lld", (long long)B);
  if (c->hop_samples != WGState::kHop)
    FAIL(SDDM_ERR_SHAPE, "hop_samples %d: WaveGrad upsamples the spectrogram x300 (wavegrad.py:157-163)", c->hop_samples);
  if (N < WGState::kHop || N % WGState::kHop)
    FAIL(SDDM_ERR_SHAPE, "%lld samples is not hop_samples (300) x frames", (long long)N);
  *F = (int)(N / WGState::kHop);
  return SDDM_OK;
}

// SDDM_spectrogram.infer (model.py:212-257) with WaveGrad: spec [B][128][F], out [B][1][300 F]
static int wg_sample(sddm_ctx* c, const float* spec, int64_t B, int64_t N, uint64_t seed, int64_t row_offset, float* out,
                     float* record, int sample_inter, const float* noise, hipStream_t s) {
  WGState& d = *c->wgs;
  int F = 0;
  WG_TRY(wg_check_shape(c, B, N, &F));
  WG_TRY(wg_prepare(c, (int)B, F));
  const int T = c->T;
  float* enctab = c->warena.at<float>(d.off_enctab);
  WG_TRY(wg_enc(c, nullptr, T + 1, enctab, s));
  WG_TRY(wg_condition(c, spec, (int)B, F, s));
  InitArgs ia{};                                       // x_T = randn(B, 1, hop F) (model.py:216)
  ia.mode = 0; ia.cond = nullptr; ia.out = out; ia.total = B * N; ia.N = N; ia.T = T;
  ia.co = c->coef(); ia.seed = seed; ia.row_offset = row_offset; ia.noise = noise;
  SDDM_HIP_CHECK(launch_init_state(ia, s));
  StepParams* sp = c->warena.at<StepParams>(d.off_sp);
  SDDM_HIP_CHECK(launch_set_params(sp, T + 1, seed, row_offset, s));
  int64_t nrec = 0;
  float* eps = d.act.at<float>(d.aoff.at("eps"));
  for (int t = T; t >= 1; --t) {
    WG_TRY(wg_network(c, out, (int)B, F, enctab, 0, &sp->t, s));
    TransArgs ta{};                                    // p_transition (diffusion.py:177-190)
    ta.mode = SDDM_TR_ORIGINAL; ta.x_t = out; ta.eps = eps; ta.cond = nullptr; ta.out = out;
    ta.total = B * N; ta.N = N; ta.t = t; ta.t_dev = &sp->t; ta.co = c->coef(); ta.seed = seed; ta.row_offset = row_offset;
    ta.noise = noise; ta.noise_ld = B * N;
    SDDM_HIP_CHECK(launch_transition(ta, s));
    if (record && t % sample_inter == 0) {
      SDDM_HIP_CHECK(hipMemcpyAsync(record + nrec * B * N, out, sizeof(float) * B * N, hipMemcpyDeviceToDevice, s));
      ++nrec;
    }
  }
  return SDDM_OK;
}

// one WaveGrad forward (wavegrad.py:167-179): spec [B][128][F], audio [B][N], noise level [B] -> eps [B][N]
static int wg_forward(sddm_ctx* c, const float* spec, const float* x_t, const float* noise_level, int64_t B, int64_t N,
                      float* eps_out, hipStream_t s) {
  WGState& d = *c->wgs;
  int F = 0;
  WG_TRY(wg_check_shape(c, B, N, &F));
  WG_TRY(wg_prepare(c, (int)B, F));
  float* encb = d.act.at<float>(d.aoff.at("encb"));
  WG_TRY(wg_enc(c, noise_level, (int)B, encb, s));
  WG_TRY(wg_condition(c, spec, (int)B, F, s));
  WG_TRY(wg_network(c, x_t, (int)B, F, encb, 1, nullptr, s));
  SDDM_HIP_CHECK(hipMemcpyAsync(eps_out, d.act.at<float>(d.aoff.at("eps")), sizeof(float) * B * N, hipMemcpyDeviceToDevice, s));
  return SDDM_OK;
}
