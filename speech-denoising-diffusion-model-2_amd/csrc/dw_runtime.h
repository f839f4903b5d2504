// DiffWave path of the runtime (included by sddm_runtime.cpp after sddm_ctx): configuration,
// weight packing, workspace and the SDDM_spectrogram.infer loop (reference model/model.py:212-257,
// model/diffwave.py).  Kernels: diffwave.hip.
#pragma once

namespace sddm {
// deferred skip GEMM + output head in one launch (diffwave.hip)
hipError_t launch_dw_skip_head(int dtype, const DWSkipArgs& a, const DWOutArgs& o, hipStream_t s);
}  // namespace sddm

struct DWState {
  int C = 64, L = 30, cycle = 10, bins = 513, hop = 256, Kp = 544;
  std::map<std::string, size_t> woff;   // packed weights in ctx->warena
  size_t off_tables = 0, off_sp = 0, off_dstab = 0;
  Arena act;                            // activations of the current (B, F)
  int B = -1, F = -1;
  size_t off_mid = 0, off_up = 0, off_cond = 0, off_xa = 0, off_xb = 0, off_skip = 0, off_eps = 0, off_dsb = 0, off_z = 0;
};

// state-dict shapes of DiffWave (diffwave.py:113-131) without the noise_estimate_model. prefix
static std::map<std::string, std::vector<int64_t>> dw_param_shapes(const DWState& d) {
  const int64_t C = d.C;
  std::map<std::string, std::vector<int64_t>> s;
  s["input_projection.weight"] = {C, 1, 1};
  s["input_projection.bias"] = {C};
  s["diffusion_embedding.projection1.weight"] = {512, 128};
  s["diffusion_embedding.projection1.bias"] = {512};
  s["diffusion_embedding.projection2.weight"] = {512, 512};
  s["diffusion_embedding.projection2.bias"] = {512};
  for (const char* k : {"conv1", "conv2"}) {
    s[std::string("spectrogram_upsampler.") + k + ".weight"] = {1, 1, 3, 32};
    s[std::string("spectrogram_upsampler.") + k + ".bias"] = {1};
  }
  for (int i = 0; i < d.L; ++i) {
    const std::string p = "residual_layers." + std::to_string(i) + ".";
    s[p + "dilated_conv.weight"] = {2 * C, C, 3};
    s[p + "dilated_conv.bias"] = {2 * C};
    s[p + "diffusion_projection.weight"] = {C, 512};
    s[p + "diffusion_projection.bias"] = {C};
    s[p + "conditioner_projection.weight"] = {2 * C, d.bins, 1};
    s[p + "conditioner_projection.bias"] = {2 * C};
    s[p + "output_projection.weight"] = {C, C, 1};
    s[p + "output_projection.bias"] = {C};
    s[p + "output_residual.weight"] = {C, C, 1};
    s[p + "output_residual.bias"] = {C};
  }
  s["skip_projection.weight"] = {C, C, 1};
  s["skip_projection.bias"] = {C};
  s["output_projection.weight"] = {1, C, 1};
  s["output_projection.bias"] = {1};
  // plain attribute of DiffusionEmbedding (diffwave.py:28), optional: the facade passes torch's
  // own fp32 values; otherwise 10 ** ((k/64) * 4/63) rounded from double
  s["diffusion_embedding.embedding_vector"] = {64};
  return s;
}

static void dw_default_embedding(std::vector<float>& v) {
  v.resize(64);
  for (int k = 0; k < 64; ++k) {
    const float step = (float)k / 64.0f;
    const float e = (step * 4.0f) / 63.0f;
    v[k] = (float)std::pow(10.0, (double)e);
  }
}

static int dw_upload_weights(sddm_ctx* c) {
  DWState& d = *c->dws;
  const int dt = c->dtype;
  const size_t es = dtype_size(dt);
  auto P = [&](const std::string& k) -> const std::vector<float>& { return c->params.at(k).data; };
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
  auto add_t = [&](const std::string& name, const std::vector<float>& v) {   // compute dtype
    Blob b;
    b.bytes.assign(v.size() * es, 0);
    for (size_t i = 0; i < v.size(); ++i) store_elem(b.bytes.data(), i, v[i], dt);
    b.off = A.reserve(b.bytes.size());
    d.woff[name] = b.off;
    blobs.push_back(std::move(b));
  };
  const int C = d.C;
  add_f32("in.w", P("input_projection.weight"));
  add_f32("in.b", P("input_projection.bias"));
  add_f32("emb.w1", P("diffusion_embedding.projection1.weight"));
  add_f32("emb.b1", P("diffusion_embedding.projection1.bias"));
  add_f32("emb.w2", P("diffusion_embedding.projection2.weight"));
  add_f32("emb.b2", P("diffusion_embedding.projection2.bias"));
  {
    const Param& ev = c->params.at("diffusion_embedding.embedding_vector");
    std::vector<float> v;
    if (ev.loaded && ev.data.size() == 64) v = ev.data;
    else dw_default_embedding(v);
    add_f32("emb.vec", v);
  }
  add_f32("up.k1", P("spectrogram_upsampler.conv1.weight"));
  add_f32("up.b1", P("spectrogram_upsampler.conv1.bias"));
  add_f32("up.k2", P("spectrogram_upsampler.conv2.weight"));
  add_f32("up.b2", P("spectrogram_upsampler.conv2.bias"));
  std::vector<float> pw, pb, cw((size_t)d.L * 128 * d.Kp, 0.f), cb((size_t)d.L * 128);
  for (int i = 0; i < d.L; ++i) {
    const std::string p = "residual_layers." + std::to_string(i) + ".";
    const auto& w = P(p + "diffusion_projection.weight");
    const auto& b = P(p + "diffusion_projection.bias");
    pw.insert(pw.end(), w.begin(), w.end());
    pb.insert(pb.end(), b.begin(), b.end());
    const auto& cwi = P(p + "conditioner_projection.weight");   // [128][bins][1]
    const auto& cbi = P(p + "conditioner_projection.bias");
    for (int co = 0; co < 2 * C; ++co) {
      for (int k = 0; k < d.bins; ++k) cw[((size_t)i * 128 + co) * d.Kp + k] = cwi[(size_t)co * d.bins + k];
      cb[(size_t)i * 128 + co] = cbi[co];
    }
    // dilated conv [128][64][3] -> [128][3*64] with k = tap*64 + ci
    const auto& dw = P(p + "dilated_conv.weight");
    std::vector<float> w1((size_t)128 * 192);
    for (int co = 0; co < 2 * C; ++co)
      for (int ci = 0; ci < C; ++ci)
        for (int tap = 0; tap < 3; ++tap) w1[(size_t)co * 192 + tap * 64 + ci] = dw[((size_t)co * C + ci) * 3 + tap];
    add_t("l" + std::to_string(i) + ".w1", w1);
    add_f32("l" + std::to_string(i) + ".b1", P(p + "dilated_conv.bias"));
    // [output_residual; output_projection] [128][64]
    std::vector<float> w2((size_t)128 * 64), b2(128);
    const auto& wr = P(p + "output_residual.weight");
    const auto& wo = P(p + "output_projection.weight");
    for (int r = 0; r < C * C; ++r) { w2[r] = wr[r]; w2[C * C + r] = wo[r]; }
    const auto& br = P(p + "output_residual.bias");
    const auto& bo = P(p + "output_projection.bias");
    for (int r = 0; r < C; ++r) { b2[r] = br[r]; b2[C + r] = bo[r]; }
    add_t("l" + std::to_string(i) + ".w2", w2);
    add_f32("l" + std::to_string(i) + ".b2", b2);
  }
  {  // every layer's output_projection side by side: [64][L*64] (k = l*64 + ci), biases summed
    std::vector<float> wo((size_t)C * d.L * C), bo(C, 0.f);
    for (int i = 0; i < d.L; ++i) {
      const std::string p = "residual_layers." + std::to_string(i) + ".";
      const auto& w = P(p + "output_projection.weight");
      const auto& bb = P(p + "output_projection.bias");
      for (int co = 0; co < C; ++co) {
        for (int ci = 0; ci < C; ++ci) wo[(size_t)co * d.L * C + (size_t)i * C + ci] = w[(size_t)co * C + ci];
        bo[co] += bb[co];
      }
    }
    add_t("skip.w", wo);
    add_f32("skip.b", bo);
  }
  add_f32("emb.pw", pw);
  add_f32("emb.pb", pb);
  add_t("cond.w", cw);
  add_f32("cond.b", cb);
  add_f32("sp.w", P("skip_projection.weight"));
  add_f32("sp.b", P("skip_projection.bias"));
  add_f32("op.w", P("output_projection.weight"));
  add_f32("op.b", P("output_projection.bias"));
  d.off_tables = A.reserve(sizeof(float) * 14 * (c->T + 1));
  d.off_sp = A.reserve(64);
  d.off_dstab = A.reserve(sizeof(float) * (size_t)(c->T + 1) * d.L * C);
  c->off_tables = d.off_tables;
  SDDM_HIP_CHECK(A.commit());
  for (const auto& b : blobs) SDDM_HIP_CHECK(hipMemcpy(A.base + b.off, b.bytes.data(), b.bytes.size(), hipMemcpyHostToDevice));
  c->params_dirty = false;
  c->tables_dirty = true;
  d.B = -1;
  return SDDM_OK;
}

static int dw_prepare(sddm_ctx* c, int B, int F) {
  DWState& d = *c->dws;
  if (d.B == B && d.F == F) return SDDM_OK;
  const size_t es = dtype_size(c->dtype);
  const size_t N = (size_t)d.hop * F;
  Arena& A = d.act;
  A.reset();
  d.off_mid = A.reserve(sizeof(float) * (size_t)B * d.bins * 16 * F);
  d.off_up = A.reserve(es * (size_t)B * N * d.Kp);
  d.off_cond = A.reserve(es * (size_t)B * N * d.L * 128);
  d.off_xa = A.reserve(es * (size_t)B * N * d.C);
  d.off_xb = A.reserve(es * (size_t)B * N * d.C);
  d.off_skip = A.reserve(sizeof(float) * (size_t)B * N * d.C);
  d.off_z = A.reserve(es * (size_t)B * N * d.L * d.C);
  d.off_eps = A.reserve(sizeof(float) * (size_t)B * N);
  d.off_dsb = A.reserve(sizeof(float) * (size_t)B * d.L * d.C);
  SDDM_HIP_CHECK(A.commit());
  d.B = B;
  d.F = F;
  return SDDM_OK;
}

// step-invariant work of one call: upsampled spectrogram and every layer's conditioner
static int dw_condition(sddm_ctx* c, const float* spec, int B, int F, hipStream_t s) {
  DWState& d = *c->dws;
  const Arena& W = c->warena;
  DWUpArgs u{};
  u.spec = spec; u.mid = d.act.at<float>(d.off_mid); u.out = d.act.base + d.off_up;
  u.B = B; u.H = d.bins; u.F = F; u.Kp = d.Kp;
  u.k1 = W.at<float>(d.woff.at("up.k1")); u.b1 = W.at<float>(d.woff.at("up.b1"));
  u.k2 = W.at<float>(d.woff.at("up.k2")); u.b2 = W.at<float>(d.woff.at("up.b2"));
  SDDM_HIP_CHECK(launch_dw_upsample(c->dtype, u, s));
  DWCondArgs g{};
  g.spec = d.act.base + d.off_up; g.w = W.base + d.woff.at("cond.w"); g.bias = W.at<float>(d.woff.at("cond.b"));
  g.out = d.act.base + d.off_cond; g.B = B; g.N = d.hop * F; g.L = d.L; g.Kp = d.Kp;
  SDDM_HIP_CHECK(launch_dw_cond(c->dtype, g, s));
  return SDDM_OK;
}

// embedding rows: the whole t table (sampling) or one row per batch item (network forward)
static int dw_embed(sddm_ctx* c, const float* noise_levels, int rows, float* out, hipStream_t s) {
  DWState& d = *c->dws;
  const Arena& W = c->warena;
  DWEmbedArgs e{};
  e.noise_levels = noise_levels; e.table = W.at<float>(d.off_tables) + (size_t)3 * (c->T + 1);
  e.time_step_mode = c->noise_time_step; e.R = rows;
  e.emb_vec = W.at<float>(d.woff.at("emb.vec"));
  e.w1 = W.at<float>(d.woff.at("emb.w1")); e.b1 = W.at<float>(d.woff.at("emb.b1"));
  e.w2 = W.at<float>(d.woff.at("emb.w2")); e.b2 = W.at<float>(d.woff.at("emb.b2"));
  e.pw = W.at<float>(d.woff.at("emb.pw")); e.pb = W.at<float>(d.woff.at("emb.pb")); e.L = d.L;
  e.out = out;
  SDDM_HIP_CHECK(launch_dw_embed(e, s));
  return SDDM_OK;
}

// one DiffWave forward: audio [B][N] fp32 -> eps [B][N] fp32 (d.off_eps)
static int dw_network(sddm_ctx* c, const float* audio, int B, int F, const float* ds, int ds_per_b, int* t_dev,
                      hipStream_t s) {
  DWState& d = *c->dws;
  const Arena& W = c->warena;
  const int N = d.hop * F;
  DWInArgs in{};
  in.audio = audio; in.w = W.at<float>(d.woff.at("in.w")); in.b = W.at<float>(d.woff.at("in.b"));
  in.x = d.act.base + d.off_xa; in.total = (int64_t)B * N; in.t_dev = t_dev;
  SDDM_HIP_CHECK(launch_dw_input(c->dtype, in, s));
  for (int i = 0; i < d.L; ++i) {
    DWLayerArgs a{};
    a.x_in = d.act.base + (i % 2 ? d.off_xb : d.off_xa);
    a.x_out = d.act.base + (i % 2 ? d.off_xa : d.off_xb);
    a.z = d.act.base + d.off_z; a.first = i == 0;
    a.cond = d.act.base + d.off_cond; a.layer = i; a.L = d.L;
    a.ds = ds; a.t_dev = t_dev; a.ds_per_b = ds_per_b;
    a.w1 = W.base + d.woff.at("l" + std::to_string(i) + ".w1"); a.b1 = W.at<float>(d.woff.at("l" + std::to_string(i) + ".b1"));
    a.w2 = W.base + d.woff.at("l" + std::to_string(i) + ".w2"); a.b2 = W.at<float>(d.woff.at("l" + std::to_string(i) + ".b2"));
    a.dil = 1 << (i % d.cycle); a.N = N; a.B = B;
    SDDM_HIP_CHECK(launch_dw_layer(c->dtype, a, s));
  }
  DWSkipArgs sk{};
  sk.z = d.act.base + d.off_z; sk.w = W.base + d.woff.at("skip.w"); sk.bias = W.at<float>(d.woff.at("skip.b"));
  sk.skip = d.act.at<float>(d.off_skip); sk.B = B; sk.N = N; sk.L = d.L;
  DWOutArgs o{};
  o.skip = d.act.at<float>(d.off_skip);
  o.wsp = W.at<float>(d.woff.at("sp.w")); o.bsp = W.at<float>(d.woff.at("sp.b"));
  o.wop = W.at<float>(d.woff.at("op.w")); o.bop = W.at<float>(d.woff.at("op.b"));
  o.sqrt_layers = (float)std::sqrt((double)d.L);
  o.eps = d.act.at<float>(d.off_eps); o.total = (int64_t)B * N;
  static const bool nofuse = std::getenv("SDDM_DW_NOFUSE") != nullptr;   // A/B knob: skip rows via HBM
  if (nofuse) {
    SDDM_HIP_CHECK(launch_dw_skip(c->dtype, sk, s));
    SDDM_HIP_CHECK(launch_dw_output(o, s));
  } else {
    SDDM_HIP_CHECK(launch_dw_skip_head(c->dtype, sk, o, s));
  }
  return SDDM_OK;
}

static int dw_check_shape(sddm_ctx* c, int64_t B, int64_t N, int* F) {
  DWState& d = *c->dws;
  if (B < 1 || B > 65535) FAIL(SDDM_ERR_INVALID_ARG, "batch %lld", (long long)B);
  if (N < d.hop || N % d.hop) FAIL(SDDM_ERR_SHAPE, "%lld samples is not hop_samples (%d) x frames", (long long)N, d.hop);
  *F = (int)(N / d.hop);
  return SDDM_OK;
}

// SDDM_spectrogram.infer (model.py:212-257): spec [B][bins][F], out [B][1][hop F]
static int dw_sample(sddm_ctx* c, const float* spec, int64_t B, int64_t N, uint64_t seed, int64_t row_offset, float* out,
                     float* record, int sample_inter, const float* noise, hipStream_t s) {
  DWState& d = *c->dws;
  int F = 0;
  int r = dw_check_shape(c, B, N, &F);
  if (r) return r;
  r = dw_prepare(c, (int)B, F);
  if (r) return r;
  const int T = c->T;
  float* dstab = c->warena.at<float>(d.off_dstab);
  r = dw_embed(c, nullptr, T + 1, dstab, s);
  if (r) return r;
  r = dw_condition(c, spec, (int)B, F, s);
  if (r) return r;
  InitArgs ia{};                                       // x_T = randn(B, 1, hop F) (model.py:216)
  ia.mode = 0; ia.cond = nullptr; ia.out = out; ia.total = B * N; ia.N = N; ia.T = T;
  ia.co = c->coef(); ia.seed = seed; ia.row_offset = row_offset; ia.noise = noise;
  SDDM_HIP_CHECK(launch_init_state(ia, s));
  StepParams* sp = c->warena.at<StepParams>(d.off_sp);
  SDDM_HIP_CHECK(launch_set_params(sp, T + 1, seed, row_offset, s));
  int64_t nrec = 0;
  for (int t = T; t >= 1; --t) {
    r = dw_network(c, out, (int)B, F, dstab, 0, &sp->t, s);
    if (r) return r;
    TransArgs ta{};                                    // p_transition (diffusion.py:177-190)
    ta.mode = SDDM_TR_ORIGINAL; ta.x_t = out; ta.eps = d.act.at<float>(d.off_eps); ta.cond = nullptr; ta.out = out;
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

// one DiffWave forward (diffwave.py:133-155): spec [B][bins][F], x_t [B][1][N], noise level [B]
static int dw_forward(sddm_ctx* c, const float* spec, const float* x_t, const float* noise_level, int64_t B, int64_t N,
                      float* eps_out, hipStream_t s) {
  DWState& d = *c->dws;
  int F = 0;
  int r = dw_check_shape(c, B, N, &F);
  if (r) return r;
  r = dw_prepare(c, (int)B, F);
  if (r) return r;
  float* dsb = d.act.at<float>(d.off_dsb);
  r = dw_embed(c, noise_level, (int)B, dsb, s);
  if (r) return r;
  r = dw_condition(c, spec, (int)B, F, s);
  if (r) return r;
  r = dw_network(c, x_t, (int)B, F, dsb, 1, nullptr, s);
  if (r) return r;
  SDDM_HIP_CHECK(hipMemcpyAsync(eps_out, d.act.at<float>(d.off_eps), sizeof(float) * B * N, hipMemcpyDeviceToDevice, s));
  return SDDM_OK;
}
