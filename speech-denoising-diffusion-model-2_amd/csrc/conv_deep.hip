// Whole-K-resident 3x3 convolution for the narrow UNet levels (segment width <= 32: the 64x32 ...
// 8x4 images with 64..320 channels of UNetModified2.py:146-235), every stride-2 Downsample
// (UNetModified2.py:103-109) and the nearest-2x Upsample convs (UNetModified2.py:93-100) landing
// there, and any wide layer whose input does not fit the row-streaming kernel.
//
// These layers are small GEMMs (M = B*pixels = 512..32768, N = Cout = 64..160, K = 9*Cin up to
// 2880 + the 1x1 res_conv) whose cost is memory latency and instruction issue, not bandwidth:
// a block's time is the length of its chain of dependent memory round trips.  The kernel is
// therefore built so that a block waits on memory ONCE:
//   1. before anything waits it issues, in the order they are needed: the producer's GroupNorm
//      tile statistics + gamma / beta, the raw input halo of all input channels (+ the raw
//      ResnetBlock.res_conv input and the identity-residual tile), bias + noise embedding, and
//      the weight fragments of the wave's first D K-steps (all of its K-steps when they fit) —
//      every load unconditional (clamped addresses) and the first staging pass straight-line
//      code, so the compiler's vmcnt accounting keeps them all in flight;
//   2. finalizes GroupNorm (fp64 Chan combination, fixed order), applies GN + SiLU, resolves the
//      nearest upsample / stride-2 halo / virtual channel concat / zero padding, and writes a
//      plane-major LDS image (a plane = one 16-byte channel unit of every halo pixel; plane
//      stride = 0 mod 256 B so the ds_read_b128 lane groups of an MFMA operand never collide);
//   3. splits K (taps x 32-channel chunks, then the res_conv chunks) round-robin over the NW
//      waves; pixel fragments come from LDS, weight fragments from the register ring;
//   4. reduces the NW partial tiles through LDS in a fixed order (deterministic), adds bias +
//      noise embedding + identity residual (both parked in LDS by step 1), stores 4-channel
//      vectors, and reduces the GroupNorm statistics of the fp32 values (before the storage
//      rounding) from registers.
// NW = 8 (one block per CU, K split 8 ways) keeps a large K resident for the small late-level
// grids; NW = 4 (two blocks per CU) overlaps two blocks' round trips on the larger grids.
#include "conv_common.h"
#include "kernels.h"

namespace sddm {

struct DeepGeo { int HR, HC, HP, PLB, PLR; };

__host__ __device__ inline DeepGeo deep_geo(bool s2, int TR, int TW, int MT) {
  DeepGeo d;
  d.HR = s2 ? 2 * TR + 1 : TR + 2;
  d.HC = s2 ? 2 * TW + 1 : TW + 2;
  d.HP = d.HR * d.HC;
  d.PLB = (d.HP * 16 + 255) / 256 * 256;
  d.PLR = (MT * 16 + 255) / 256 * 256;
  return d;
}

// LDS byte layout of one block; region 0 (the staged image) is reused for the partial tiles
struct DeepLds { int rres, badd, gsc, total; };

template <typename T, int MT, int NW, int NB>
__host__ __device__ inline DeepLds deep_layout(const DeepGeo& g, int nck, int rck, int Cin, bool ident) {
  constexpr int ES = (int)sizeof(T), UPP = 2 * ES, NBP = NB + 4;
  constexpr int SLOTS = (NW == 8 && MT >= 128) ? 4 : NW;   // two-stage reduction for 8 x 128 pixels
  const int red = SLOTS * MT * NBP * 4;
  const int stage = nck * UPP * g.PLB + rck * UPP * g.PLR;
  DeepLds L;
  int off = stage > red ? stage : red;
  L.rres = off;
  off += ident ? MT * NB * ES : 0;
  L.badd = off;
  off += 32 * 4;
  L.gsc = off;
  off += 2 * Cin * 4;
  L.total = off;
  return L;
}

// Chan merge of (n, mean, M2) partial statistics
__device__ __forceinline__ void chan_merge(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  const float nt = n + nb;
  if (nb == 0.f) return;
  if (n == 0.f) { n = nb; mean = meanb; m2 = m2b; return; }
  const float d = meanb - mean;
  mean += d * (nb / nt);
  m2 += m2b + d * d * (n * nb / nt);
  n = nt;
}

// Activation loads.  HO (hand-off mode, the team kernel below): the bytes were stored by another
// workgroup of this launch on the same XCD, so they are read from that XCD's L2 past this CU's L1
// (which may still hold stale lines of the same addresses): buffer_load ... sc1 over the lane
// arena `hb` (conv_common.h ho_rsrc).
template <bool HO>
__device__ __forceinline__ f32x4 ld_act(const f32x4* p, const char* hb) {
  if constexpr (HO)
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(ho_rsrc(hb), (unsigned)((const char*)p - hb), 0, 16));
  else return *p;
}

struct NoWait {
  __device__ __forceinline__ void operator()() const {}
};

// The noise-embedding row of a conv (ResnetBlock.noise_func): table [rows][ld], the row is the
// step counter *t_dev (sampling) or the image (network forward, per_b); tab == null: none
struct TembRef { const float* tab; int ld; const int* t_dev; int per_b; };

// One output tile (TR x TW pixels of image b, output channels [zb NB, zb NB + NB)) of the
// whole-K-resident convolution.  `wait` runs after the weight fragments are issued and before
// any activation is loaded (team kernel: the dependency poll; per-layer kernel: nothing).
template <typename T, bool S2, int MT, int NW, int D, int NB, bool HO, typename Wait>
__device__ __forceinline__ void deep_tile(const ConvArgs& a, const TembRef& te, int tile, int b, int zb, char* smem,
                                          const Wait& wait, const char* hb = nullptr,
                                          unsigned long long* hst = nullptr) {
  constexpr int NT = 64 * NW;
  constexpr int ES = (int)sizeof(T);
  constexpr int UPP = 2 * ES;          // 16-byte planes per 32-channel chunk
  constexpr int UPL = ES / 2;          // planes per MFMA lane group (8 channels)
  constexpr int VE = 16 / ES;          // channels per plane
  constexpr int FP = MT / 16, FC = NB / 16, NBP = NB + 4;
  constexpr int TPP = NB / 4;          // epilogue threads per pixel (4 channels each)
  constexpr int UPR = NB * ES / 16;    // 16-byte units of one pixel's identity-residual channels
  static_assert(NB == 16 || NB == 32, "16 or 32 output channels per block");
  constexpr int MAXU = ES == 4 ? (NW == 8 ? 6 : 8) : (NW == 8 ? 10 : 16);   // units per thread per pass
  constexpr int SLOTS = (NW == 8 && MT >= 128) ? 4 : NW;

  int tid = threadIdx.x;
  // team kernel: an opaque copy per item, so the per-thread index math of the staging units is
  // recomputed inside the ticket loop instead of being hoisted out of it and kept live (spilled)
  if constexpr (HO) asm volatile("" : "+v"(tid));
  const int lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  const int n0 = zb * NB;
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  const int y0 = ty * a.TR, x0 = tx * a.TW;
  const int npv = a.TR * a.TW;         // valid pixels (< MT only for images smaller than a tile)
  const DeepGeo geo = deep_geo(S2, a.TR, a.TW, MT);
  const int HC = geo.HC, HP = geo.HP, PLB = geo.PLB, PLR = geo.PLR;
  const int Cin = a.CA + a.CB, nck = Cin / 32;
  const int RC = a.RCA + a.RCB, rck = a.res_mode == 2 ? RC / 32 : 0;
  const bool gn = a.gamma != nullptr, ident = a.res_mode == 1;
  const DeepLds lay = deep_layout<T, MT, NW, NB>(geo, nck, rck, Cin, ident);
  float* gsc = (float*)(smem + lay.gsc);                 // [2][Cin] GroupNorm scale / shift
  const int res_off = nck * UPP * PLB;
  const int img_in = a.Hi * a.Wi, img_out = a.Ho * a.Wo;
  const T* srcA = (const T*)a.srcA + (size_t)b * img_in * a.CA;
  const T* srcB = a.CB ? (const T*)a.srcB + (size_t)b * img_in * a.CB : srcA;
  const T* rawA = a.res_mode == 2 ? (const T*)a.rawA + (size_t)b * img_out * a.RCA : srcA;
  const T* rawB = (a.res_mode == 2 && a.RCB) ? (const T*)a.rawB + (size_t)b * img_out * a.RCB : rawA;
  const T* rsrc = ident ? (const T*)a.res_src + (size_t)b * img_out * a.Cout + n0 : srcA;
  SDDM_STAMP(a, 0);

  // this wave's K steps (wave-uniform) and the first D weight fragments of each
  const int ns3 = nck * 9, ns = ns3 + rck;
  const int nj = wv < ns ? (ns - wv + NW - 1) / NW : 0;
  const int s_last = wv + NW * max(nj - 1, 0);
  // weights in MFMA-fragment order (ConvArgs::wgt_f): the 64 lanes of one A fragment read one
  // contiguous 1 KiB (bf16 / f16) or 2 KiB (fp32) run, not 16 rows x 64 B pieces
  const int cb0 = n0 / 16;
  const T* wbase = (const T*)a.wgt_f + (size_t)lane * 8;
  const T* rbase = (const T*)a.res_wgt_f + (size_t)lane * 8;
  auto wfrag = [&](int s, int fc) -> Frag<T> {
    const T* p = s < ns3 ? wbase + ((size_t)(cb0 + fc) * ns3 + s) * 512
                         : rbase + ((size_t)(cb0 + fc) * rck + (s - ns3)) * 512;
    return load_frag<T>((const char*)p);
  };
  Frag<T> wa[D][FC];
  auto issue_weights = [&]() {
#pragma unroll
    for (int d = 0; d < D; ++d)
#ifdef SDDM_DEEP_GUARD
      if (d < nj)                                        // wave-uniform
#endif
      {
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) wa[d][fc] = (a.dbg & 32) ? Frag<T>{} : wfrag(min(wv + NW * d, s_last), fc);
      }
  };
  // hand-off mode: the weights (never written in the launch) stream in while the dependency is awaited
  if constexpr (HO) issue_weights();
  wait();

  // ---------------- 1. issue every load of the block ----------------
  GNLoad gl;
  const GNFuse gf{a.gstA, a.gtilesA, a.gntileA, a.gstB, a.gtilesB, a.gntileB, a.gamma, a.beta, a.groups, a.eps};
  gl.template issue<HO>(gf, b, a.CA, a.CB, gn, a.bias, hb);

  // staging units: [0, n3) halo planes (8 lanes = 8 consecutive halo pixels of one plane),
  // [n3, n3 + nres) raw res_conv input at the output pixels, then the identity-residual tile
  const int nq3 = nck * UPP;
  const int n3 = (HP + 7) / 8 * 8 * nq3;
  const int nqr = rck * UPP;
  const int nres = nqr * MT;
  const int total = n3 + nres + (ident ? MT * UPR : 0);
  const float rnq3 = 1.0f / (float)max(nq3, 1), rnqr = 1.0f / (float)max(nqr, 1);
  const float rHC = 1.0f / (float)HC, rTW = 1.0f / (float)a.TW;
  // packed destination: LDS byte offset << 10 | (GroupNorm channel + 2); -2 = zero, -1 = raw copy
  auto unit = [&](int u, f32x4& r, int& pk) {
    const T* ptr = srcA;               // any valid address; the value is unused when pk < 0
    int d = -1, gs = -1;
    if (u < n3) {
      const int grp = u >> 3, gq = fdivi(grp, rnq3), q = grp - gq * nq3, hp = gq * 8 + (u & 7);
      const int hy = fdivi(hp, rHC), hx = hp - hy * HC;
      int iy, ix;
      bool ok;
      if (S2) {
        iy = 2 * y0 - 1 + hy; ix = 2 * x0 - 1 + hx;
        ok = iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi;
      } else {
        iy = y0 - 1 + hy; ix = x0 - 1 + hx;
        ok = iy >= 0 && iy < a.Ho && ix >= 0 && ix < a.Wo;
        if (a.upsample) { iy >>= 1; ix >>= 1; }
      }
      const int c = q * VE;
      const bool fromA = c < a.CA;
      if (ok) ptr = (fromA ? srcA : srcB) + (iy * a.Wi + ix) * (fromA ? a.CA : a.CB) + (fromA ? c : c - a.CA);
      if (hp < HP) { d = q * PLB + hp * 16; gs = ok ? c : -2; }
    } else if (u < n3 + nres) {
      const int v = u - n3, grp = v >> 3, gq = fdivi(grp, rnqr), q = grp - gq * nqr, p = gq * 8 + (v & 7);
      d = res_off + q * PLR + p * 16;
      gs = -2;
      if (p < npv) {
        const int py = fdivi(p, rTW), px = p - py * a.TW;
        const int c = q * VE;
        const bool fromA = c < a.RCA;
        ptr = (fromA ? rawA : rawB) + ((y0 + py) * a.Wo + (x0 + px)) * (fromA ? a.RCA : a.RCB) +
              (fromA ? c : c - a.RCA);
        gs = -1;
      }
    } else if (u < total) {            // identity residual [p][NB channels]
      const int v = u - n3 - nres, p = v / UPR, q = v - p * UPR;
      d = lay.rres + v * 16;
      gs = -2;
      if (p < npv) {
        const int py = fdivi(p, rTW), px = p - py * a.TW;
        ptr = rsrc + ((y0 + py) * a.Wo + (x0 + px)) * a.Cout + q * VE;
        gs = -1;
      }
    }
    r = ld_act<HO>((const f32x4*)ptr, hb);
    pk = d < 0 ? -1 : (d << 10) | (gs + 2);
  };
  auto commit = [&](const f32x4& r, int pk) {
    if (pk < 0) return;
    const int gs = (pk & 1023) - 2;
    f32x4 v = r;
    if (gs == -2) v = f32x4{0.f, 0.f, 0.f, 0.f};
    else if (gn && gs >= 0 && !(a.dbg & 2)) v = transform_lds<T>(v, gsc + gs, gsc + Cin + gs);
    *(f32x4*)(smem + (pk >> 10)) = v;
  };
  // the first pass: nu0 (block-uniform) units per thread; a uniform branch skips the rest
  const int nu0 = min((total + NT - 1) / NT, MAXU);
  f32x4 reg[MAXU];
  int pk[MAXU];
#pragma unroll
  for (int k = 0; k < MAXU; ++k) {
#ifdef SDDM_DEEP_GUARD
    pk[k] = -1;
    if (k < nu0)
#endif
    unit(tid + k * NT, reg[k], pk[k]);
    if (a.dbg & 4) pk[k] = -1;
  }

  // the step counter selecting the noise-embedding row (loaded with everything else; the
  // bias + embedding loads that depend on it are issued after the staging wait)
  const int t_now = te.t_dev ? *te.t_dev : 0;

  if constexpr (!HO) issue_weights();
  SDDM_STAMP(a, 1);

  // ---------------- 2. GroupNorm finalize, GN + SiLU into the LDS image ----------------
  if (gn && !(a.dbg & 1)) gl.template finish<HO>(gf, b, a.CA, a.CB, gsc, gsc + Cin, hb);
  lds_sync();                                            // scale / shift visible (loads stay in flight)
  SDDM_STAMP(a, 2);
  if (HO && hst && wv == 0) hst[0] = __builtin_amdgcn_s_memrealtime();   // team stamps (experiments)
#pragma unroll
  for (int k = 0; k < MAXU; ++k)
#ifdef SDDM_DEEP_GUARD
    if (k < nu0)
#endif
    commit(reg[k], pk[k]);
  for (int u0 = MAXU * NT; u0 < total; u0 += MAXU * NT) {   // inputs larger than one pass
#pragma unroll
    for (int k = 0; k < MAXU; ++k) unit(u0 + tid + k * NT, reg[k], pk[k]);
#pragma unroll
    for (int k = 0; k < MAXU; ++k) commit(reg[k], pk[k]);
  }
  lds_sync();
  SDDM_STAMP(a, 3);
  if (HO && hst && wv == 0) hst[1] = __builtin_amdgcn_s_memrealtime();
  // bias + noise embedding of this thread's 4 epilogue channels: in flight during the K loop
  const int ec4 = (tid & (TPP - 1)) * 4;
  float bb[4], sshift;
  {
    const float* trow = te.tab ? te.tab + (size_t)(te.per_b ? b : t_now) * te.ld : a.bias;
#pragma unroll
    for (int i = 0; i < 4; ++i) {                        // unconditional loads (no wait at a join)
      const float bv = a.bias[n0 + ec4 + i], tv = trow[n0 + ec4 + i];
      bb[i] = bv + (te.tab ? tv : 0.f);
    }
    const int cs = n0 + (tid & (NB - 1));                // statistics shift of channel n0 + tid (tid < NB)
    const float sbv = a.bias[cs], stv = trow[cs];
    sshift = sbv + (te.tab ? stv : 0.f);
  }

  // ---------------- 3. this wave's K steps ----------------
  int pix_off[FP];
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    int p = fp * 16 + (lane & 15);
    if (p >= npv) p = 0;
    const int py = p / a.TW, px = p - py * a.TW;
    pix_off[fp] = S2 ? ((2 * py) * HC + 2 * px) * 16 : (py * HC + px) * 16;
  }
  f32x4 acc[FP][FC];
#pragma unroll
  for (int i = 0; i < FP; ++i)
#pragma unroll
    for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nj_run = (a.dbg & 8) ? 0 : nj;
  for (int j0 = 0; j0 < nj_run; j0 += D) {
    const bool refill = j0 + D < nj;                     // the ring wraps (K longer than D steps)
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int j = j0 + d;
      const int s = wv + NW * j;
      if (j < nj) {
        Frag<T> bf[FP];
        if (s < ns3) {
          const int lc = s / 9, tap = s - 9 * lc, dy = tap / 3, dx = tap - 3 * dy;
          const char* pb = smem + (lc * UPP + g * UPL) * PLB + (dy * HC + dx) * 16;
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) bf[fp] = load_planes<T>(pb + pix_off[fp], PLB);
        } else {
          const char* pb = smem + res_off + ((s - ns3) * UPP + g * UPL) * PLR + (lane & 15) * 16;
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) bf[fp] = load_planes<T>(pb + fp * 256, PLR);
        }
#pragma unroll
        for (int fc = 0; fc < FC; ++fc)
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) mfma_frag(acc[fp][fc], wa[d][fc], bf[fp]);
      }
      if (refill) {
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) wa[d][fc] = wfrag(min(s + NW * D, s_last), fc);
      }
    }
  }
  SDDM_STAMP(a, 4);
  if (HO && hst && wv == 0) hst[2] = __builtin_amdgcn_s_memrealtime();

  // ---------------- 4. reduce the partial tiles: red[slot][MT][NBP] ----------------
  lds_sync();                                       // every wave is done with the image
  float* red = (float*)smem;
  auto put = [&](int slot) {
#pragma unroll
    for (int fp = 0; fp < FP; ++fp) {
      const int p = fp * 16 + (lane & 15);
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) *(f32x4*)(red + (slot * MT + p) * NBP + fc * 16 + 4 * g) = acc[fp][fc];
    }
  };
  if (SLOTS < NW) {                                      // waves 4..7 into slots, waves 0..3 add theirs
    if (wv >= SLOTS) put(wv - SLOTS);
    lds_sync();
    if (wv < SLOTS) {
#pragma unroll
      for (int fp = 0; fp < FP; ++fp) {
        const int p = fp * 16 + (lane & 15);
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) acc[fp][fc] += *(const f32x4*)(red + (wv * MT + p) * NBP + fc * 16 + 4 * g);
      }
      put(wv);
    }
  } else {
    put(wv);
  }
  lds_sync();

  constexpr int PPI = NT / TPP;                          // pixels per epilogue pass
  constexpr int EIT = (MT + PPI - 1) / PPI;
  float sn = 0.f, s1[4], s2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { s1[i] = 0.f; s2[i] = 0.f; }
  T* out = (T*)a.out + (size_t)b * img_out * a.Cout + n0 + ec4;
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int p = it * PPI + tid / TPP;
    if (p < npv) {
      const int py = fdivi(p, rTW), px = p - py * a.TW;
      f32x4 s = *(const f32x4*)(red + p * NBP + ec4);
#pragma unroll
      for (int w = 1; w < SLOTS; ++w) s += *(const f32x4*)(red + (w * MT + p) * NBP + ec4);
      float d[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) d[i] = s[i];
      if (ident) {
        const T* rp = (const T*)(smem + lay.rres) + p * NB + ec4;
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] += to_f32<T>(rp[i]);
      }
      store4<T>(out + ((y0 + py) * a.Wo + (x0 + px)) * a.Cout, d[0] + bb[0], d[1] + bb[1], d[2] + bb[2], d[3] + bb[3]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {                    // sums about the shift bb (the same for
        s1[i] += d[i];                                 // every thread of a channel: they add)
        s2[i] += d[i] * d[i];
      }
      sn += 1.f;
    }
  }
  SDDM_STAMP(a, 5);
  if (a.stats && !(a.dbg & 16)) {
    // the lanes of a DPP row holding the same 4 channels (16 / TPP of them, TPP apart) add by
    // row rotations, then the 4 rows of every wave through LDS, summed by one thread per channel
    auto rowred = [](float x) {
      if constexpr (TPP == 4) x += dpp_f32<0x124>(x);   // row_ror:4
      return x + dpp_f32<0x128>(x);                    // row_ror:8
    };
    const float tn = rowred(sn);
    float t1[4], t2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { t1[i] = rowred(s1[i]); t2[i] = rowred(s2[i]); }
    lds_sync();                                        // red reads done
    float* xs = red;                                   // [NW * 4 rows][NB channels][3]
    if ((lane & 15) < TPP)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float* e = xs + ((wave * 4 + (lane >> 4)) * NB + ec4 + i) * 3;
        e[0] = tn; e[1] = t1[i]; e[2] = t2[i];
      }
    lds_sync();
    if (tid < NB) {
      float n = 0.f, u1 = 0.f, u2 = 0.f;
#pragma unroll 4
      for (int r = 0; r < NW * 4; ++r) {
        const float* e = xs + (r * NB + tid) * 3;
        n += e[0]; u1 += e[1]; u2 += e[2];
      }
      const float shift = sshift;
      float* dst = a.stats + (((size_t)b * a.n_tiles + tile) * a.Cout + n0 + tid) * 2;
      dst[0] = (shift + u1 / n) * n;
      dst[1] = fmaxf(u2 - u1 * u1 / n, 0.f);
    }
  }
  SDDM_STAMP(a, 6);
  if (HO && hst && wv == 0) hst[3] = __builtin_amdgcn_s_memrealtime();
  SDDM_STAMP(a, 7);
}

// One launch per layer: one tile per block, in the XCD-aware block order.
template <typename T, bool S2, int MT, int NW, int D, int NB>
__global__ __launch_bounds__(64 * NW, 8 / NW) void conv_deep_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int tile, b, zb;
  xcd_block(a.n_tiles, a.Cout / NB, tile, b, zb);
  const TembRef te{a.temb, a.temb_ld, a.t_dev, a.temb_per_b};
  deep_tile<T, S2, MT, NW, D, NB, false>(a, te, tile, b, zb, smem, NoWait{});
}

// ---------------------------------------------------------------------------------------------
// Deep-level team kernel: a run of consecutive convolutions (the UNet levels whose images are a
// few hundred pixels: Downsample -> ResnetBlocks -> mid -> ResnetBlocks -> Upsample, the loop
// bodies of UNetModified2.py:252-265) as ONE launch.  Per-layer launches of these layers are
// each a chain of dependent memory round trips after a kernel boundary (L2 written back and
// invalidated, HBM latency for every first load); here the images never leave the L2 of the XCD
// that works on them:
//   * image b belongs to the team of XCD b % 8; a workgroup reads its XCD from HW_REG_XCC_ID and
//     serves that team, so producer and consumer of every hand-off share one L2 whatever the
//     dispatcher's placement;
//   * a team's work is a ticket queue in op-major order (op, image, tile x channel block); a
//     workgroup takes the next ticket, issues the item's weight fragments (constant in the
//     launch), then polls the per-(op, image) completion counter of the op it reads from, reads
//     the activations, GroupNorm statistics and residuals past its L1 (ld_act<true>) and computes
//     exactly the per-layer kernel's tile (same tiling, same arithmetic: bit-identical outputs);
//   * completion: every wave drains its stores (s_waitcnt vmcnt(0): the stores reached the L2),
//     workgroup barrier, one lane adds 1 to the counter (an L2 atomic of this XCD).
// Tickets are taken in dependency order, so the lowest unfinished ticket never waits on an
// unclaimed one: no co-residency is assumed and the queue cannot deadlock.  Spins are bounded
// (s_memrealtime); a timeout sets the error word and the workgroup carries on.
// ---------------------------------------------------------------------------------------------
// variant index: s2 * 6 + mt_index(32, 64, 128) * 2 + (nb == 32)
__host__ __device__ constexpr int team_var(bool s2, int mt, int nb) {
  return (s2 ? 6 : 0) + (mt == 32 ? 0 : mt == 64 ? 1 : 2) * 2 + (nb == 32 ? 1 : 0);
}

template <typename T, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void conv_team_kernel(TeamArgs ta, const TeamOp* __restrict__ ops) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ int s_ticket;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  xcc &= 7;
  const int B = ta.B;
  const int nimg = (int)xcc < B ? (B - 1 - (int)xcc) / 8 + 1 : 0;
  if (nimg == 0) return;
  // every counter on a 256-byte slot of its own (pollers of one counter do not queue behind
  // another's traffic): ticket of team x at slot x, done[op][b] at slot 8 + op * B + b
  unsigned* ticket = ta.ctr + xcc * kTeamSlot;
  unsigned* done = ta.ctr + 8 * kTeamSlot;
  // Only wave-uniform branches around the barriers of this loop: a lane-0 branch (ticket, poll,
  // publish) gets structurised into a lane-divergent loop around the barriers, which hangs (measured).
  // Wave 0 takes the ticket (its lane 0 adds 1), polls and publishes.
  const bool w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
  const unsigned one = (threadIdx.x & 63) == 0 ? 1u : 0u;
  for (;;) {
    if (w0)
      s_ticket = (int)__builtin_amdgcn_readfirstlane(
          __hip_atomic_fetch_add(ticket, one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    __syncthreads();
    int t = __builtin_amdgcn_readfirstlane(s_ticket);   // uniform: the op table is read through SGPRs
    const int tk = t;
    unsigned long long* hst = ta.stamps && tk < 4096 ? ta.stamps + ((size_t)xcc * 4096 + tk) * 8 + 4 : nullptr;
    const unsigned long long ts0 = ta.stamps ? __builtin_amdgcn_s_memrealtime() : 0ull;
    unsigned long long ts1 = 0;
    int op = 0;
    for (; op < ta.nops; ++op) {                         // scalar walk over the op table
      const int n = nimg * ops[op].items;
      if (t < n) break;
      t -= n;
    }
    if (op >= ta.nops) break;
    const TeamOp& o = ops[op];
    const int j = t / o.items, item = t - j * o.items;
    const int b = (int)xcc + 8 * j;
    const int zb = item / o.a.n_tiles, tile = item - zb * o.a.n_tiles;
    const TembRef te{o.toff >= 0 ? ta.temb + o.toff : nullptr, ta.temb_ld, ta.t_dev, ta.temb_per_b};
    const int dep = o.dep;
    auto wait = [&]() {
      if (dep >= 0) {
        if (w0) {                                        // wave-uniform (scalar) poll loop
          const unsigned need = (unsigned)ops[dep].items;
          unsigned* c = done + (dep * B + b) * kTeamSlot;
          const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
          for (unsigned spins = 0;; ++spins) {
            const unsigned v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (v >= need) break;
            __builtin_amdgcn_s_sleep(4);                 // ~0.1 us between polls
            // 20 ms (100 MHz clock) or 2^20 polls: give up, flag it
            if (spins > (1u << 20) || __builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {
              __hip_atomic_store(ta.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
          }
        }
        asm volatile("s_barrier" ::: "memory");          // orders the activation loads after the poll
      }
      if (ta.stamps) ts1 = __builtin_amdgcn_s_memrealtime();
    };
    switch (o.var) {
#define SDDM_TEAM_CASE(S2V, MTV, NBV)                                                                  \
  case team_var(S2V, MTV, NBV):                                                                        \
    deep_tile<T, S2V, MTV, NW, 8, NBV, true>(o.a, te, tile, b, zb, smem, wait, ta.arena, hst);                         \
    break;
      SDDM_TEAM_CASE(false, 32, 16) SDDM_TEAM_CASE(false, 32, 32) SDDM_TEAM_CASE(false, 64, 16)
      SDDM_TEAM_CASE(false, 64, 32) SDDM_TEAM_CASE(false, 128, 16) SDDM_TEAM_CASE(false, 128, 32)
      SDDM_TEAM_CASE(true, 32, 16) SDDM_TEAM_CASE(true, 32, 32) SDDM_TEAM_CASE(true, 64, 16)
      SDDM_TEAM_CASE(true, 64, 32)
#undef SDDM_TEAM_CASE
      default: break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // every wave: its stores reached the L2
    __syncthreads();
    if (w0) __hip_atomic_fetch_add(done + (op * B + b) * kTeamSlot, one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ta.stamps && w0 && tk < 4096) {                  // (every lane of wave 0 stores the same words)
      unsigned long long* st = ta.stamps + ((size_t)xcc * 4096 + tk) * 8;
      st[0] = (unsigned long long)op | ((unsigned long long)b << 16);
      st[1] = ts0; st[2] = ts1; st[3] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// weight-ring depth for a wave's K steps: the whole K when it fits in the register budget
template <typename T, int MT, int NW>
static int deep_ring(int steps_per_wave) {
  if (sizeof(T) == 4 || NW == 4) return 8 / (int)(sizeof(T) == 4 ? 2 : 1);
  if (steps_per_wave <= 8 || MT >= 128) return 8;
  return 12;
}

template <typename T, bool S2, int MT, int NW, int NB>
static hipError_t deep_go(const ConvArgs& a, int B, hipStream_t s, size_t* lo) {
  const int nck = (a.CA + a.CB) / 32, rck = a.res_mode == 2 ? (a.RCA + a.RCB) / 32 : 0;
  const DeepGeo geo = deep_geo(S2, a.TR, a.TW, MT);
  const DeepLds lay = deep_layout<T, MT, NW, NB>(geo, nck, rck, a.CA + a.CB, a.res_mode == 1);
  if (lo) {
    *lo = (size_t)lay.total;
    return hipSuccess;
  }
  if (a.TR * a.TW > MT || a.Cout % NB || (a.CA + a.CB) % 32 || (a.CA + a.CB) > 1000 || (a.RCA + a.RCB) % 32)
    return hipErrorInvalidValue;
  if (lay.total > kLdsBytes) return hipErrorInvalidValue;
  const dim3 grid = xcd_grid(a.n_tiles, B, a.Cout / NB), blk(64 * NW);
  const int D = deep_ring<T, MT, NW>((nck * 9 + rck + NW - 1) / NW);
#define SDDM_RING(DV)                                                                         \
  if (D == DV) {                                                                              \
    hipLaunchKernelGGL((conv_deep_kernel<T, S2, MT, NW, DV, NB>), grid, blk, lay.total, s, a); \
    return hipGetLastError();                                                                 \
  }
  if constexpr (sizeof(T) == 4) {
    SDDM_RING(4)
  } else if constexpr (NW == 4 || MT >= 128) {
    SDDM_RING(8)
  } else {
    SDDM_RING(8) SDDM_RING(12)
  }
#undef SDDM_RING
  return hipErrorInvalidValue;
}

// nb: output channels per block (32, or 16 for twice the blocks with half the weights each)
template <typename T>
static hipError_t deep_dispatch(int mt, int nw, int nb, bool s2, const ConvArgs& a, int B, hipStream_t s, size_t* lo) {
#define SDDM_DEEP(S2V, MTV, NWV, NBV) \
  if (s2 == S2V && mt == MTV && nw == NWV && nb == NBV) return deep_go<T, S2V, MTV, NWV, NBV>(a, B, s, lo);
  SDDM_DEEP(false, 32, 4, 32) SDDM_DEEP(false, 64, 4, 32) SDDM_DEEP(false, 128, 4, 32)
  SDDM_DEEP(true, 32, 4, 32) SDDM_DEEP(true, 64, 4, 32) SDDM_DEEP(true, 128, 4, 32)
  SDDM_DEEP(false, 32, 8, 32) SDDM_DEEP(false, 64, 8, 32) SDDM_DEEP(false, 128, 8, 32)
  SDDM_DEEP(true, 32, 8, 32) SDDM_DEEP(true, 64, 8, 32) SDDM_DEEP(true, 128, 8, 32)
  SDDM_DEEP(false, 16, 4, 16) SDDM_DEEP(false, 32, 4, 16) SDDM_DEEP(false, 64, 4, 16) SDDM_DEEP(false, 128, 4, 16)
  SDDM_DEEP(true, 16, 4, 16) SDDM_DEEP(true, 32, 4, 16) SDDM_DEEP(true, 64, 4, 16)
  SDDM_DEEP(false, 32, 8, 16) SDDM_DEEP(false, 64, 8, 16) SDDM_DEEP(false, 128, 8, 16)
#undef SDDM_DEEP
  if (lo) *lo = (size_t)1 << 40;
  return hipErrorInvalidValue;
}

hipError_t launch_conv_deep(int dtype, int mt, bool s2, const ConvArgs& a, int B, hipStream_t s) {
  const int nw = a.deep_nw, nb = a.deep_nb ? a.deep_nb : 32;
  if (dtype == DT_F32) return deep_dispatch<float>(mt, nw, nb, s2, a, B, s, nullptr);
  if (dtype == DT_BF16) return deep_dispatch<bf16_t>(mt, nw, nb, s2, a, B, s, nullptr);
  return deep_dispatch<f16_t>(mt, nw, nb, s2, a, B, s, nullptr);
}

int conv_deep_ring_depth(int dtype, int mt, int nw, int ksteps) {
  const int spw = (ksteps + nw - 1) / nw;
  if (dtype == DT_F32) return 4;
  if (nw == 4 || mt >= 128) return 8;
  return deep_ring<bf16_t, 64, 8>(spw);
}

int conv_team_var(bool s2, int mt, int nb) {
  if ((mt != 32 && mt != 64 && mt != 128) || (nb != 16 && nb != 32) || (s2 && mt == 128)) return -1;
  return team_var(s2, mt, nb);
}

// (8-wave items only: the 4-wave variant measured slower, 438 vs 414 us per step)
hipError_t launch_conv_team(int dtype, int nw, const TeamArgs& a, int lds_bytes, int blocks, hipStream_t s) {
  if (dtype == DT_F32 || lds_bytes > team_lds_budget(nw) || a.nops < 1 || blocks < 8 || nw != 8)
    return hipErrorInvalidValue;
  if (dtype == DT_BF16) hipLaunchKernelGGL((conv_team_kernel<bf16_t, 8>), dim3(blocks), dim3(512), lds_bytes, s, a, a.ops);
  else hipLaunchKernelGGL((conv_team_kernel<f16_t, 8>), dim3(blocks), dim3(512), lds_bytes, s, a, a.ops);
  return hipGetLastError();
}

size_t conv_deep_lds_bytes(int dtype, int mt, bool s2, const ConvArgs& a) {
  size_t lo = (size_t)1 << 40;
  const int nw = a.deep_nw, nb = a.deep_nb ? a.deep_nb : 32;
  if (dtype == DT_F32) (void)deep_dispatch<float>(mt, nw, nb, s2, a, 1, 0, &lo);
  else if (dtype == DT_BF16) (void)deep_dispatch<bf16_t>(mt, nw, nb, s2, a, 1, 0, &lo);
  else (void)deep_dispatch<f16_t>(mt, nw, nb, s2, a, 1, 0, &lo);
  return lo;
}

}  // namespace sddm
