// K-streamed implicit-GEMM 3x3 convolution for the middle and deep UNet levels (bf16 / f16):
// Block / ResnetBlock convs, stride-2 Downsample and nearest-2x Upsample convs
// (UNetModified2.py:93-142).  GEMM M = output pixels of one image tile, N = a block of NB output
// channels, K = 9 taps x Cin, plus the 1x1 ResnetBlock.res_conv (UNetModified2.py:135) as extra
// K chunks.
//
// Why this shape (measured on the whole-K kernel conv_deep.hip, which it replaces where it wins):
// there a block of 32 output channels staged the GroupNorm + SiLU of its whole input halo, so the
// transform of every input element ran Cout/32 times, and each wave pulled its weight fragments
// as 16 rows x 64 B pieces.  Here
//   * a block owns NB = 32..96 output channels, so an input element is transformed once per
//     channel block (once per pixel for most layers), and up to 256 output pixels, so the weights
//     a block streams are reused by that many pixels;
//   * K runs in 32-channel chunks through a two-deep pipeline with one barrier per chunk: while
//     the MFMAs of chunk k run, the raw input halo of chunk k+1 and its weights (pre-packed
//     chunk-major in ConvArgs::wgt_t: every wave-instruction reads one contiguous 1 KiB run)
//     stream into registers; after the MFMAs the same waves apply GroupNorm + SiLU to chunk k+1
//     and write its operand image and weight chunk to LDS (round 5: the weights had gone by
//     LDS-DMA, whose per-unit issue cost made the chunk loop slower, SDDM_TILE_WREG);
//   * 8-wave blocks keep two waves per SIMD, so one wave's VALU transform overlaps the other's
//     MFMAs.
// LDS operand images are plane-major (a plane = 8 channels, 16 B per pixel or output channel);
// the pixel slot is XOR-swizzled by 2*plane so the staging writes (4 planes of 2 pixels per
// 8-lane group) are conflict-free while any 16 consecutive slots of one plane still map to 16
// distinct bank groups for the ds_read_b128 MFMA operand reads.  Stride-2 halos store even and
// odd columns in separate halves so the taps of consecutive output pixels read consecutive slots.
// Epilogue: bias + noise embedding + residual (identity, or the res_conv chunks), 4 channels per
// lane stored as T, and GroupNorm tile statistics of the fp32 values (before the storage
// rounding) as shifted sums reduced with DPP row adds, in the format every conv kernel consumes.
#include "conv_common.h"
#include "conv_tile_cfg.h"
#include "kernels.h"

#ifndef SDDM_TILE_WREG
// 1: weight chunks through registers + ds_write_b128 (default; one global load and one LDS store
// per 16-byte unit issue cheaper than one LDS-DMA per unit: tile launches -3..-8 us per step,
// bench +1 %); 0: by LDS-DMA (A/B builds)
#define SDDM_TILE_WREG 1
#endif

namespace sddm {

template <typename T, bool S2, int WPX, int WCO, int FP, int FC, int MAXU, int SH>
__global__ __launch_bounds__(64 * WPX * WCO) void conv_tile_kernel(ConvArgs a) {
  constexpr int NWV = WPX * WCO, NT = 64 * NWV;
  constexpr int MT = WPX * FP * 16, NB = WCO * FC * 16;
  constexpr int WCH = 576 * NB;                            // LDS bytes of one 3x3 weight chunk
  static_assert(sizeof(T) == 2, "conv_tile is the 16-bit path");
  typedef T vec4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // layer geometry: compile-time for a specialised shape (SH > 0, kTileShapes), else the arguments
  constexpr ConvShape SC = kTileShapes[SH];
  constexpr bool CS = SH > 0;
  SDDM_SHAPE_GEO(SC, CS, S2, a)

  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, c16 = lane & 15, q = lane & 3;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wp = wv % WPX, wc = wv / WPX;
  int tile, b, zb;
  xcd_block<SDDM_XCD_ZIN != 0>(gNT, gCout / NB, tile, b, zb);
  const int n0 = zb * NB;
  const int ty = tile / gTX, tx = tile - ty * gTX;
  const int y0 = ty * gTR, x0 = tx * gTW;
  const int npv = gTR * gTW;                             // valid pixels (< MT: image smaller than a tile)
  const int Cin = gCA + gCB, nck = Cin / 32, ckA = gCA / 32;
  const int RC = gRCA + gRCB, rck = gRes == 2 ? RC / 32 : 0, rckA = gRCA / 32;
  const int nk = nck + rck;
  const bool gn = gGN, ident = gRes == 1;
  const TileGeo geo = tile_geo(S2, gTR, gTW, MT, rck > 0);
  const int HC = geo.HC, HE = geo.HE, PLB = geo.PLB;
  const int nbuf = nk > 1 ? 2 : 1;                         // double buffers only when K streams
  char* IB = smem;                                         // [nbuf][4 planes][PLB] operand images
  char* WB = IB + nbuf * geo.ibb;                          // [nbuf][WCH]           weight chunks
  float* gsc = (float*)(WB + nbuf * WCH);                  // [2][Cin]              GroupNorm scale / shift
  const float rHC = 1.0f / (float)HC, rTW = 1.0f / (float)gTW;
  const int img_in = gHi * gWi, img_out = gHo * gWo;
  const T* srcA = (const T*)a.srcA + (size_t)b * img_in * gCA;
  const T* srcB = gCB ? (const T*)a.srcB + (size_t)b * img_in * gCB : srcA;
  const T* rawA = rck ? (const T*)a.rawA + (size_t)b * img_out * gRCA : srcA;
  const T* rawB = (rck && gRCB) ? (const T*)a.rawB + (size_t)b * img_out * gRCB : rawA;
  SDDM_STAMP(a, 0);

  // ---------------- prologue: every independent load before anything waits ----------------
  GNLoad gl;
  const GNFuse gf{a.gstA, a.gtilesA, a.gntileA, a.gstB, a.gtilesB, a.gntileB, a.gamma, a.beta, a.groups, a.eps};
  gl.issue(gf, b, gCA, gCB, gn, a.bias);
  const int t_now = a.t_dev ? *a.t_dev : 0;
  const float* trow = a.temb ? a.temb + (size_t)(a.temb_per_b ? b : t_now) * a.temb_ld : a.bias;
  const int cw0 = wc * FC * 16, pw0 = wp * FP * 16;
  float bb[FC][4];
#pragma unroll
  for (int fc = 0; fc < FC; ++fc)
#pragma unroll
    for (int i = 0; i < 4; ++i) {                          // unconditional loads (no wait at a join)
      const int co = n0 + cw0 + fc * 16 + 4 * g + i;
      const float bv = a.bias[co], tv = trow[co];
      bb[fc][i] = bv + (a.temb ? tv : 0.f);
    }
  float sshift;                                            // statistics shift of channel n0 + tid (tid < NB)
  {
    const int cs = n0 + (tid % NB);
    const float bv = a.bias[cs], tv = trow[cs];
    sshift = bv + (a.temb ? tv : 0.f);
  }
  // this lane's output pixels (MFMA column c16 of each pixel fragment)
  int ppy[FP], ppx[FP];
  bool pok[FP];
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    int p = pw0 + fp * 16 + c16;
    pok[fp] = p < npv;
    if (!pok[fp]) p = 0;
    ppy[fp] = fdivi(p, rTW);
    ppx[fp] = p - ppy[fp] * gTW;
  }
  vec4 r1[FP][FC];                                         // identity residual (res_conv = Identity)
  {
    const T* rs = ident ? (const T*)a.res_src + (size_t)b * img_out * gCout : srcA;
#pragma unroll
    for (int fp = 0; fp < FP; ++fp) {
      const int po = ident ? ((y0 + ppy[fp]) * gWo + (x0 + ppx[fp])) * gCout : 0;
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) r1[fp][fc] = *(const vec4*)(rs + po + (ident ? n0 + cw0 + fc * 16 + 4 * g : 0));
    }
  }
  // staging geometry of this thread's 3x3 units (the same for every chunk): unit u = tid + j NT
  // is plane q = u & 3 of halo slot u >> 2; source pixel (-1: zero padding), swizzled LDS offset
  // (-1: past the halo)
  int spx[MAXU], sof[MAXU];
#pragma unroll
  for (int j = 0; j < MAXU; ++j) {
    const int u = tid + j * NT, s = u >> 2;
    const int hy = fdivi(s, rHC), hx = s - hy * HC;
    int iy, ix, slot;
    bool ok;
    if (S2) {
      iy = 2 * y0 - 1 + hy; ix = 2 * x0 - 1 + hx;
      ok = iy >= 0 && iy < gHi && ix >= 0 && ix < gWi;
      slot = hy * HC + ((hx & 1) ? HE + (hx >> 1) : (hx >> 1));
    } else {
      iy = y0 - 1 + hy; ix = x0 - 1 + hx;
      ok = iy >= 0 && iy < gHo && ix >= 0 && ix < gWo;
      if (gUp) { iy >>= 1; ix >>= 1; }
      slot = s;
    }
    spx[j] = ok ? iy * gWi + ix : -1;
    sof[j] = u < geo.nu3 ? q * PLB + ((slot ^ (q << 1)) << 4) : -1;
  }

  // raw chunk k -> registers (unconditional loads at clamped addresses)
  f32x4 rr[MAXU];
  auto load_raw = [&](int k) {
    if (k < nck) {
      const bool fa = k < ckA;
      const T* base = (fa ? srcA + k * 32 : srcB + (k - ckA) * 32) + q * 8;
      const int cs = fa ? gCA : gCB;
#pragma unroll
      for (int j = 0; j < MAXU; ++j) rr[j] = *(const f32x4*)(base + (spx[j] < 0 ? 0 : spx[j] * cs));
    } else {                                               // res_conv chunk: raw input at the output pixels
      const int r = k - nck;
      const bool fa = r < rckA;
      const T* base = (fa ? rawA + r * 32 : rawB + (r - rckA) * 32) + q * 8;
      const int cs = fa ? gRCA : gRCB;
#pragma unroll
      for (int j = 0; j < MAXU; ++j) {
        const int p = (tid + j * NT) >> 2;
        const int py = fdivi(p, rTW), px = p - py * gTW;
        rr[j] = *(const f32x4*)(base + (p < npv ? ((y0 + py) * gWo + (x0 + px)) * cs : 0));
      }
    }
  };
  // weight chunk k -> WB[buf]: one contiguous run of NB units per (tap, plane)
  auto issue_w = [&](int k, int buf) {
    char* dst = WB + buf * WCH;
    const bool res = k >= nck;
    const int nw = (res ? 4 : 36) * NB;
    const char* ws = res ? (const char*)a.res_wgt_t + (size_t)(k - nck) * 4 * gCout * 16
                         : (const char*)a.wgt_t + (size_t)k * 36 * gCout * 16;
    for (int u0 = wv * 64; u0 < nw; u0 += NT) {
      const int u = u0 + lane, r = u / NB, co = u - r * NB;
      glds16(ws + ((size_t)r * gCout + n0 + co) * 16, dst + u0 * 16);
    }
  };
  // weight chunk k through registers (WR): WU 16-byte units per thread, loaded with the raw halo
  // at the top of an iteration and written to WB[buf] after the MFMAs, beside the transform.  The
  // generic (runtime-geometry) instantiations with more than 6 accumulator fragments per wave keep
  // LDS-DMA: the extra registers made them spill (config #5's 256-pixel x 96-channel tiles)
  constexpr bool WR = SDDM_TILE_WREG && (SH > 0 || FP * FC <= 6);
  constexpr int WU = (36 * NB + NT - 1) / NT;
  f32x4 wr[WR ? WU : 1];
  auto load_w = [&](int k) {
    const bool res = k >= nck;
    const int nw = (res ? 4 : 36) * NB;
    const char* ws = res ? (const char*)a.res_wgt_t + (size_t)(k - nck) * 4 * gCout * 16
                         : (const char*)a.wgt_t + (size_t)k * 36 * gCout * 16;
#pragma unroll
    for (int i = 0; i < WU; ++i) {
      const int u = tid + i * NT, uu = u < nw ? u : 0, r = uu / NB, co = uu - r * NB;
      wr[i] = *(const f32x4*)(ws + ((size_t)r * gCout + n0 + co) * 16);
    }
  };
  auto store_w = [&](int k, int buf) {
    const int nw = (k >= nck ? 4 : 36) * NB;
    char* dst = WB + buf * WCH;
#pragma unroll
    for (int i = 0; i < WU; ++i) {
      const int u = tid + i * NT;
      if (u < nw) *(f32x4*)(dst + u * 16) = wr[i];
    }
  };
  // chunk k: registers -> IB[buf] with zero padding and GroupNorm + SiLU (3x3 chunks of a Block)
  auto transform = [&](int k, int buf) {
    char* ib = IB + buf * geo.ibb;
    if (k < nck) {
      float sc[8], sh[8];
      if (gn) {
        const int c = k * 32 + q * 8;
#pragma unroll
        for (int j = 0; j < 8; j += 4) {
          const f32x4 s4 = *(const f32x4*)(gsc + c + j), h4 = *(const f32x4*)(gsc + Cin + c + j);
#pragma unroll
          for (int i = 0; i < 4; ++i) { sc[j + i] = s4[i]; sh[j + i] = h4[i]; }
        }
      }
#pragma unroll
      for (int j = 0; j < MAXU; ++j) {
        if (sof[j] < 0) continue;
        f32x4 v = rr[j];
        if (spx[j] < 0) v = f32x4{0.f, 0.f, 0.f, 0.f};
        else if (gn) v = transform_regs<T>(v, sc, sh);
        *(f32x4*)(ib + sof[j]) = v;
      }
    } else {
#pragma unroll
      for (int j = 0; j < MAXU; ++j) {
        const int u = tid + j * NT, p = u >> 2;
        if (u >= geo.nur) continue;
        f32x4 v = rr[j];
        if (p >= npv) v = f32x4{0.f, 0.f, 0.f, 0.f};
        *(f32x4*)(ib + q * PLB + ((p ^ (q << 1)) << 4)) = v;
      }
    }
  };

  f32x4 acc[FP][FC];
#pragma unroll
  for (int i = 0; i < FP; ++i)
#pragma unroll
    for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // slot of tap (0, 0) for each pixel fragment of this lane
  int sbase[FP];
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) sbase[fp] = S2 ? 2 * ppy[fp] * HC + ppx[fp] : ppy[fp] * HC + ppx[fp];
  const int gx = g << 1;
  auto mma = [&](int k, int buf) {
    const char* ib = IB + buf * geo.ibb + g * PLB;
    const char* wb = WB + buf * WCH + (g * NB + cw0 + c16) * 16;
    if (k < nck) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3, dx = tap - 3 * dy;
        const int toff = S2 ? dy * HC + (dx == 0 ? 0 : (dx == 1 ? HE : 1)) : dy * HC + dx;
        Frag<T> bf[FP];
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) bf[fp] = load_frag<T>(ib + (((sbase[fp] + toff) ^ gx) << 4));
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) {
          const Frag<T> af = load_frag<T>(wb + (tap * 4 * NB + fc * 16) * 16);
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) mfma_frag(acc[fp][fc], af, bf[fp]);
        }
      }
    } else {
      Frag<T> bf[FP];
#pragma unroll
      for (int fp = 0; fp < FP; ++fp) {
        const int p = pok[fp] ? pw0 + fp * 16 + c16 : 0;
        bf[fp] = load_frag<T>(ib + ((p ^ gx) << 4));
      }
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) {
        const Frag<T> af = load_frag<T>(wb + fc * 16 * 16);
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) mfma_frag(acc[fp][fc], af, bf[fp]);
      }
    }
  };

  load_raw(0);
  if constexpr (WR) load_w(0);
  else issue_w(0, 0);
  if (gn) gl.finish(gf, b, gCA, gCB, gsc, gsc + Cin);
  SDDM_STAMP(a, 1);
  __syncthreads();                                         // gsc visible
  transform(0, 0);
  if constexpr (WR) {
    store_w(0, 0);
    lds_sync();
  } else {
    dma_sync();                                            // operand image 0, weights 0 (LDS-DMA)
  }
  SDDM_STAMP(a, 2);
#ifdef SDDM_STAMPS
  // timing ablations of the profiling build (SDDM_STAMPS_DBG): 4 no raw loads, 32 no weight DMA,
  // 8 no MFMAs, 2 no staging transform, 128 no output stores (results are garbage)
  const int dbg = a.dbg;
#else
  constexpr int dbg = 0;
#endif
  for (int k = 0; k < nk; ++k) {
    const int cur = k & 1, nxt = cur ^ 1;
    if constexpr (WR) {
      if (k + 1 < nk) {
        if (!(dbg & 4)) load_raw(k + 1);                   // in flight during the MFMAs
        if (!(dbg & 32)) load_w(k + 1);
      }
      if (!(dbg & 8)) mma(k, cur);
      if (k + 1 < nk) {
        if (!(dbg & 2)) transform(k + 1, nxt);             // IB[nxt] / WB[nxt] were read by chunk k - 1
        if (!(dbg & 32)) store_w(k + 1, nxt);
      }
      lds_sync();
    } else {
      if (k + 1 < nk) {
        if (!(dbg & 4)) load_raw(k + 1);                   // in flight during the MFMAs
        if (!(dbg & 32)) issue_w(k + 1, nxt);              // WB[nxt] was read by chunk k - 1
      }
      if (!(dbg & 8)) mma(k, cur);
      if (k + 1 < nk && !(dbg & 2)) transform(k + 1, nxt); // IB[nxt] was read by chunk k - 1
      dma_sync();                                          // WB[nxt] landed by LDS-DMA from every wave
    }
  }
  SDDM_STAMP(a, 4);

  // ---------------- epilogue ----------------
  T* out = (T*)a.out + (size_t)b * img_out * gCout;
  float s1[FC][4], s2[FC][4], nl = 0.f;
#pragma unroll
  for (int fc = 0; fc < FC; ++fc)
#pragma unroll
    for (int i = 0; i < 4; ++i) { s1[fc][i] = 0.f; s2[fc][i] = 0.f; }
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    if (!pok[fp]) continue;
    nl += 1.f;
    const int po = ((y0 + ppy[fp]) * gWo + (x0 + ppx[fp])) * gCout;
#pragma unroll
    for (int fc = 0; fc < FC; ++fc) {
      const int co = n0 + cw0 + fc * 16 + 4 * g;
      float d[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) d[i] = acc[fp][fc][i] + (ident ? to_f32<T>(r1[fp][fc][i]) : 0.f);
      if (!(dbg & 128)) store4<T>(out + po + co, d[0] + bb[fc][0], d[1] + bb[fc][1], d[2] + bb[fc][2], d[3] + bb[fc][3]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {                        // sums about the shift bb (stable)
        s1[fc][i] += d[i];
        s2[fc][i] += d[i] * d[i];
      }
    }
  }
  SDDM_STAMP(a, 5);
  if (a.stats) {
    // every lane of a channel uses the same shift, so the shifted sums add directly: the 16
    // pixel lanes of a DPP row, then the WPX pixel waves through LDS
    float* red = (float*)IB;                               // [WPX][NB][3] (operand images are dead)
    const float nr = row_sum16(nl);
#pragma unroll
    for (int fc = 0; fc < FC; ++fc)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float t1 = row_sum16(s1[fc][i]), t2 = row_sum16(s2[fc][i]);
        if (c16 == 0) {
          float* e = red + (wp * NB + cw0 + fc * 16 + 4 * g + i) * 3;
          e[0] = nr; e[1] = t1; e[2] = t2;
        }
      }
    lds_sync();
    if (tid < NB) {
      float n = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < WPX; ++w) {
        const float* e = red + (w * NB + tid) * 3;
        n += e[0]; t1 += e[1]; t2 += e[2];
      }
      const int co = tid;
      const float mean = sshift + t1 / n;
      float* dst = a.stats + (((size_t)b * gNT + tile) * gCout + n0 + co) * 2;
      dst[0] = mean * n;
      dst[1] = fmaxf(t2 - t1 * t1 / n, 0.f);
    }
  }
  SDDM_STAMP(a, 6);
  SDDM_STAMP(a, 7);
}

template <int I>
static size_t tile_lds_cfg(bool s2, const ConvArgs& a) {
  constexpr TileCfgX c = kTileCfgs[I];
  constexpr int MT = c.wpx * c.fp * 16, NB = c.wco * c.fc * 16;
  const TileGeo g = tile_geo(s2, a.TR, a.TW, MT, a.res_mode == 2);
  const int NT = 64 * c.wpx * c.wco, maxu = s2 ? c.maxu_s2 : c.maxu;
  if (g.nu3 > maxu * NT || g.nur > maxu * NT) return (size_t)1 << 40;   // more staging units than registers
  const int nk = (a.CA + a.CB) / 32 + (a.res_mode == 2 ? (a.RCA + a.RCB) / 32 : 0);
  return (size_t)tile_lds(g, NB, a.CA + a.CB, nk > 1 ? 2 : 1);
}

template <typename T, bool S2, int I, int SH = 0>
static hipError_t tile_go(const ConvArgs& a, int B, hipStream_t s) {
  constexpr TileCfgX c = kTileCfgs[I];
  constexpr int MT = c.wpx * c.fp * 16, NB = c.wco * c.fc * 16;
  const size_t lds = tile_lds_cfg<I>(S2, a);
  if (a.TR * a.TW > MT || a.Cout % NB || (a.CA + a.CB) % 32 || a.CA % 32 || (a.RCA + a.RCB) % 32 || a.RCA % 32 ||
      lds > kLdsBytes || !a.wgt_t || (a.res_mode == 2 && !a.res_wgt_t))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL((conv_tile_kernel<T, S2, c.wpx, c.wco, c.fp, c.fc, S2 ? c.maxu_s2 : c.maxu, SH>),
                     xcd_grid(a.n_tiles, B, a.Cout / NB), dim3(64 * c.wpx * c.wco), lds, s, a);
  return hipGetLastError();
}

// the specialised shapes SH = 1 .. kNTileShapes-1 whose configuration, stride and geometry match
template <typename T, bool S2, int SH>
static bool tile_shape_go(int cfg, const ConvArgs& a, int B, hipStream_t s, hipError_t& e) {
  if constexpr (SH >= kNTileShapes) {
    return false;
  } else {
    constexpr ConvShape c = kTileShapes[SH];
    if constexpr (c.s2 == (S2 ? 1 : 0) && shape_for_type<T>(c)) {
      if (c.cfg == cfg && conv_shape_geo_matches(c, S2, a)) { e = tile_go<T, S2, c.cfg, SH>(a, B, s); return true; }
    }
    return tile_shape_go<T, S2, SH + 1>(cfg, a, B, s, e);
  }
}

template <typename T, bool S2>
static hipError_t tile_dispatch(int cfg, const ConvArgs& a, int B, hipStream_t s) {
  static const bool generic = std::getenv("SDDM_NO_TILE_SHAPES") != nullptr;   // A/B runs
  hipError_t e;
  if (!generic && tile_shape_go<T, S2, 1>(cfg, a, B, s, e)) return e;
  switch (cfg) {
#define SDDM_TILE(I) \
  case I: return tile_go<T, S2, I>(a, B, s);
    SDDM_TILE(0) SDDM_TILE(1) SDDM_TILE(2) SDDM_TILE(3) SDDM_TILE(4) SDDM_TILE(5)
    SDDM_TILE(6) SDDM_TILE(7) SDDM_TILE(8) SDDM_TILE(9) SDDM_TILE(10) SDDM_TILE(11) SDDM_TILE(12)
#undef SDDM_TILE
    default: return hipErrorInvalidValue;
  }
}

int conv_tile_ncfg() { return kNTileCfgs; }
TileCfg conv_tile_cfg(int cfg) {
  const TileCfgX& c = kTileCfgs[cfg];
  return TileCfg{c.wpx, c.wco, c.fp, c.fc};
}

hipError_t launch_conv_tile(int dtype, int cfg, bool s2, const ConvArgs& a, int B, hipStream_t s) {
  if (dtype == DT_BF16) return s2 ? tile_dispatch<bf16_t, true>(cfg, a, B, s) : tile_dispatch<bf16_t, false>(cfg, a, B, s);
  if (dtype == DT_F16) return s2 ? tile_dispatch<f16_t, true>(cfg, a, B, s) : tile_dispatch<f16_t, false>(cfg, a, B, s);
  return hipErrorInvalidValue;
}

size_t conv_tile_lds_bytes(int cfg, bool s2, const ConvArgs& a) {
  switch (cfg) {
#define SDDM_TILE(I) \
  case I: return tile_lds_cfg<I>(s2, a);
    SDDM_TILE(0) SDDM_TILE(1) SDDM_TILE(2) SDDM_TILE(3) SDDM_TILE(4) SDDM_TILE(5)
    SDDM_TILE(6) SDDM_TILE(7) SDDM_TILE(8) SDDM_TILE(9) SDDM_TILE(10) SDDM_TILE(11) SDDM_TILE(12)
#undef SDDM_TILE
    default: return (size_t)1 << 40;
  }
}

}  // namespace sddm
