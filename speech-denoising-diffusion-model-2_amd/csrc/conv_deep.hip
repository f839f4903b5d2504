// Whole-K-resident 3x3 convolution for the narrow UNet levels (segment width <= 32: the 64x32 ...
// 8x4 images with 64..320 channels of UNetModified2.py:146-235), every stride-2 Downsample
// (UNetModified2.py:103-109) and the nearest-2x Upsample convs (UNetModified2.py:93-100) landing
// there, and any wide layer whose input does not fit the row-streaming kernel.
//
// These layers are small GEMMs (M = B*pixels = 512..32768, N = Cout = 64..160, K = 9*Cin up to
// 2880 + the 1x1 res_conv).  A block moves 30-300 KB and runs a handful of MFMAs per wave, so
// its time is the number of instructions each wave issues between its phases, not bandwidth:
// the round-4 kernel spent ~2300 instructions per wave computing staging addresses (one
// branchy unit at a time, ten units per thread whether the halo needed them or not) and ~3500
// more transforming them, for 12 MFMAs (round-5 stamps).  This kernel:
//   1. issues everything before anything waits: the raw input halo by LDS-DMA straight into the
//      plane-major operand image (one wave-instruction = 64 halo pixels of one 16-byte channel
//      plane; each lane's pixel offset is computed ONCE and reused for every plane; pixels
//      outside the image read a zero page), the raw res_conv input the same way, the producer's
//      GroupNorm tile statistics, the weight fragments of the wave's first D K-steps and the
//      identity-residual tile (registers);
//   2. finalizes GroupNorm (fp32 Chan combination of the producer's tile statistics, fixed
//      order) into per-channel scale / shift in LDS;
//   3. applies GroupNorm + SiLU in place, one 64-pixel x 16-byte chunk per lane per step, the
//      plane's scale / shift wave-uniform (zero-padded pixels stay zero: the reference pads the
//      activated tensor, UNetModified2.py:116-120);
//   4. splits K (taps x 32-channel chunks, then the res_conv chunks) round-robin over the NW
//      waves; pixel fragments come from LDS, weight fragments from the register ring;
//   5. reduces the NW partial tiles through LDS in a fixed order (deterministic), adds bias +
//      noise embedding + identity residual, stores 4-channel vectors and the GroupNorm tile
//      statistics of the fp32 values (before the storage rounding).
// NW = 8 (one block per CU, K split 8 ways) keeps a large K resident for the small late-level
// grids; NW = 4 (two blocks per CU) overlaps two blocks on the larger grids.
#include "conv_common.h"
#include "conv_tile_cfg.h"
#include "kernels.h"

namespace sddm {

// 16 zero bytes for the halo pixels outside the image (LDS-DMA has no zero fill)
__device__ __attribute__((aligned(256))) unsigned char g_deep_zero[256];

constexpr int kDeepMaxChunks = 10;   // 64-pixel chunks of a halo plane (640 halo pixels)

// phase stamps: the default set (1 all issued, 2 GroupNorm landed, 3 operand image written, 4 K
// loop, 5 stored, 6 statistics) or, with -DSDDM_STAMPS_ISSUE, a finer split of the issue phase (1
// weights issued, 2 staging loads issued, 3 all issued, 4 GroupNorm landed, 5 image written, 6 K loop)
#ifdef SDDM_STAMPS_ISSUE
#define DS_W(a) SDDM_STAMP(a, 1)
#define DS_STG(a) SDDM_STAMP(a, 2)
#define DS_ISSUED(a) SDDM_STAMP(a, 3)
#define DS_LANDED(a) SDDM_STAMP(a, 4)
#define DS_XFORM(a) SDDM_STAMP(a, 5)
#define DS_KLOOP(a) SDDM_STAMP(a, 6)
#define DS_STORED(a) do {} while (0)
#define DS_STATS(a) do {} while (0)
#else
#define DS_W(a) do {} while (0)
#define DS_STG(a) do {} while (0)
#define DS_ISSUED(a) SDDM_STAMP(a, 1)
#define DS_LANDED(a) SDDM_STAMP(a, 2)
#define DS_XFORM(a) SDDM_STAMP(a, 3)
#define DS_KLOOP(a) SDDM_STAMP(a, 4)
#define DS_STORED(a) SDDM_STAMP(a, 5)
#define DS_STATS(a) SDDM_STAMP(a, 6)
#endif

// timing ablations of the profiling build (SDDM_STAMPS_DBG; results are garbage under any flag):
// 32 no weight loads
#ifdef SDDM_STAMPS
#define SDDM_DEEP_DBG(bit) ((a.dbg & (bit)) != 0)
#else
#define SDDM_DEEP_DBG(bit) false
#endif

struct DeepGeo { int HR, HC, HP, NCH, PLB, NCR, PLR; };

__host__ __device__ inline DeepGeo deep_geo(bool s2, int TR, int TW, int MT) {
  DeepGeo d;
  d.HR = s2 ? 2 * TR + 1 : TR + 2;
  d.HC = s2 ? 2 * TW + 1 : TW + 2;
  d.HP = d.HR * d.HC;
  d.NCH = (d.HP + 63) / 64;            // one LDS-DMA wave-instruction per 64 pixels of a plane
  d.PLB = d.NCH * 1024;                // plane stride (0 mod 256 B: conflict-free operand reads)
  d.NCR = (MT + 63) / 64;
  d.PLR = d.NCR * 1024;
  return d;
}

// LDS byte layout of one block; region 0 (the staged image) is reused for the partial tiles
struct DeepLds { int gsc, total; };

template <typename T, int MT, int NW, int NB>
__host__ __device__ inline DeepLds deep_layout(const DeepGeo& g, int Cin, int RC) {
  constexpr int VE = 16 / (int)sizeof(T), NBP = NB + 4;
  constexpr int SLOTS = (NW == 8 && MT >= 128) ? 4 : NW;   // two-stage reduction for 8 x 128 pixels
  const int red = SLOTS * MT * NBP * 4;
  const int stage = (Cin / VE) * g.PLB + (RC / VE) * g.PLR;
  DeepLds L;
  L.gsc = stage > red ? stage : red;
  L.total = L.gsc + 2 * Cin * 4;
  return L;
}

// GroupNorm items per thread: 64 (tile, channel) statistics per group in one round trip
template <int NW> struct DeepGN { static constexpr int GK = NW == 8 ? 4 : 8; };

// deep kernel shapes (conv_tile_cfg.h ConvShape; cfg = pixels per tile): UNetModified2
// config_unet.json at 16448 samples with the measured per-layer kernels of configs/conv_tuning.json
static constexpr ConvShape kDeepShapes[] = {
    {-1, 0, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},   // generic (fields unused)
    // generated by tools/gen_shapes.py from configs/conv_tuning.json (do not edit by hand)
    {32, 1, 2, 16, 32, 16, 96, 0, 96, 0, 0, 0, 0, 0, 4, 32, 0},  // downs.6
    {128, 0, 8, 16, 32, 16, 96, 0, 128, 0, 0, 0, 1, 0, 8, 32, 0},  // downs.7.block1
    {128, 0, 8, 16, 32, 16, 128, 0, 128, 96, 0, 2, 1, 0, 8, 32, 0},  // downs.7.block2
    {32, 1, 4, 8, 16, 8, 128, 0, 128, 0, 0, 0, 0, 0, 4, 32, 0},  // downs.8
    {64, 0, 8, 8, 16, 8, 128, 0, 160, 0, 0, 0, 1, 0, 4, 32, 0},  // downs.9.block1
    {64, 0, 8, 8, 16, 8, 160, 0, 160, 128, 0, 2, 1, 0, 4, 32, 0},  // downs.9.block2
    {32, 1, 8, 4, 8, 4, 160, 0, 160, 0, 0, 0, 0, 0, 4, 16, 0},  // downs.10
    {32, 0, 8, 4, 8, 4, 160, 0, 160, 0, 0, 0, 1, 0, 8, 16, 0},  // mid.0.block1
    {32, 0, 8, 4, 8, 4, 160, 0, 160, 0, 0, 1, 1, 0, 8, 16, 0},  // mid.0.block2
    {32, 0, 8, 4, 8, 4, 160, 160, 160, 0, 0, 0, 1, 0, 8, 16, 0},  // ups.0.block1
    {32, 0, 8, 4, 8, 4, 160, 0, 160, 160, 160, 2, 1, 0, 8, 16, 0},  // ups.0.block2
    {64, 0, 8, 8, 16, 8, 160, 0, 160, 0, 0, 0, 0, 1, 4, 32, 0},  // ups.1
    {32, 0, 4, 8, 16, 8, 160, 160, 128, 0, 0, 0, 1, 0, 8, 32, 0},  // ups.2.block1
    {32, 0, 4, 8, 16, 8, 128, 0, 128, 160, 160, 2, 1, 0, 4, 32, 0},  // ups.2.block2
    {32, 0, 4, 8, 16, 8, 128, 128, 128, 0, 0, 0, 1, 0, 8, 32, 0},  // ups.3.block1
    {32, 0, 4, 8, 16, 8, 128, 0, 128, 128, 128, 2, 1, 0, 4, 32, 0},  // ups.3.block2
    {128, 0, 8, 16, 32, 16, 128, 0, 128, 0, 0, 0, 0, 1, 4, 32, 0},  // ups.4
    {128, 0, 8, 16, 32, 16, 128, 128, 96, 0, 0, 0, 1, 0, 8, 32, 0},  // ups.5.block1
    {128, 0, 8, 16, 32, 16, 96, 0, 96, 128, 128, 2, 1, 0, 8, 32, 0},  // ups.5.block2
    {128, 0, 8, 16, 32, 16, 96, 96, 96, 0, 0, 0, 1, 0, 8, 32, 0},  // ups.6.block1
    {128, 0, 8, 16, 32, 16, 96, 0, 96, 96, 96, 2, 1, 0, 4, 32, 0},  // ups.6.block2
    {64, 1, 4, 16, 64, 16, 96, 0, 96, 0, 0, 0, 0, 0, 4, 32, 1},  // c5:downs.6
    {64, 0, 8, 8, 32, 8, 128, 0, 160, 0, 0, 0, 1, 0, 4, 32, 1},  // c5:downs.9.block1
    {64, 0, 8, 8, 32, 8, 160, 0, 160, 128, 0, 2, 1, 0, 4, 32, 1},  // c5:downs.9.block2
    {32, 1, 8, 4, 16, 4, 160, 0, 160, 0, 0, 0, 0, 0, 4, 32, 1},  // c5:downs.10
    {32, 0, 8, 4, 16, 4, 160, 0, 160, 0, 0, 0, 1, 0, 4, 32, 1},  // c5:mid.0.block1
    {32, 0, 8, 4, 16, 4, 160, 0, 160, 0, 0, 1, 1, 0, 4, 32, 1},  // c5:mid.0.block2
    {32, 0, 8, 4, 16, 4, 160, 160, 160, 0, 0, 0, 1, 0, 4, 32, 1},  // c5:ups.0.block1
    {32, 0, 8, 4, 16, 4, 160, 0, 160, 160, 160, 2, 1, 0, 4, 32, 1},  // c5:ups.0.block2
    {64, 0, 8, 8, 32, 8, 160, 0, 160, 0, 0, 0, 0, 1, 4, 32, 1},  // c5:ups.1
};
static constexpr int kNDeepShapes = (int)(sizeof(kDeepShapes) / sizeof(kDeepShapes[0]));

// One output tile (TR x TW pixels of image b, output channels [zb NB, zb NB + NB)).
template <typename T, bool S2, int MT, int NW, int D, int NB, int SH>
__global__ __launch_bounds__(64 * NW, 8 / NW) void conv_deep_kernel(ConvArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // layer geometry: compile-time for a specialised shape (SH > 0, kDeepShapes), else the arguments
  constexpr ConvShape SC = kDeepShapes[SH];
  constexpr bool CS = SH > 0;
  SDDM_SHAPE_GEO(SC, CS, S2, a)
  constexpr int NT = 64 * NW;
  constexpr int ES = (int)sizeof(T);
  constexpr int UPP = 2 * ES;          // 16-byte planes per 32-channel chunk
  constexpr int UPL = ES / 2;          // planes per MFMA lane group (8 channels)
  constexpr int VE = 16 / ES;          // channels per plane
  constexpr int FP = MT / 16, FC = NB / 16, NBP = NB + 4;
  constexpr int TPP = NB / 4;          // epilogue threads per pixel (4 channels each)
  constexpr int PPI = NT / TPP;        // pixels per epilogue pass
  constexpr int EIT = (MT + PPI - 1) / PPI;
  static_assert(NB == 16 || NB == 32 || NB == 64, "16, 32 or 64 output channels per block");
  constexpr int SLOTS = (NW == 8 && MT >= 128) ? 4 : NW;

  int tile, b, zb;
  if (a.deep_zin) xcd_block<true>(gNT, gCout / NB, tile, b, zb);
  else xcd_block<false>(gNT, gCout / NB, tile, b, zb);
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n0 = zb * NB;
  const int ty = tile / gTX, tx = tile - ty * gTX;
  const int y0 = ty * gTR, x0 = tx * gTW;
  const int npv = gTR * gTW;         // valid pixels (< MT only for images smaller than a tile)
  const DeepGeo geo = deep_geo(S2, gTR, gTW, MT);
  const int HC = geo.HC, PLB = geo.PLB, PLR = geo.PLR;
  const int Cin = gCA + gCB, nck = Cin / 32, npl = Cin / VE, plA = gCA / VE;
  const int RC = gRes == 2 ? gRCA + gRCB : 0, rck = RC / 32, nplr = RC / VE, plRA = gRCA / VE;
  const bool gn = gGN, ident = gRes == 1;
  const DeepLds lay = deep_layout<T, MT, NW, NB>(geo, Cin, RC);
  float* gsc = (float*)(smem + lay.gsc);                 // [2][Cin] GroupNorm scale / shift
  const int res_off = npl * PLB;
  const int img_in = gHi * gWi, img_out = gHo * gWo;
  const char* srcA = (const char*)a.srcA + (size_t)b * img_in * gCA * ES;
  const char* srcB = (const char*)(gCB ? a.srcB : a.srcA) + (size_t)b * img_in * gCB * ES;
  const char* zero = (const char*)g_deep_zero;
  // the step counter selecting the noise-embedding row: an unconditional scalar load (a
  // conditional one is waited for at its branch join, in front of every load below)
  const int* tdp = a.t_dev ? a.t_dev : (const int*)g_deep_zero;
  const int t_step = *tdp;
  const int t_now = a.temb_per_b ? b : t_step;
  SDDM_STAMP(a, 0);

  // ---------------- 1. issue every load of the block ----------------
  const int ec4 = (tid & (TPP - 1)) * 4;
  // (a) GroupNorm tile statistics of the producer(s) (issued even for a conv without GroupNorm:
  // unconditional loads, no wait at a branch join)
  GNLoadT<DeepGN<NW>::GK> gl;
  const GNFuse gf{a.gstA, a.gtilesA, a.gntileA, a.gstB, a.gtilesB, a.gntileB, a.gamma, a.beta, a.groups, a.eps};
  gl.issue(gf, b, gCA, gCB, gn, a.bias);
  // (b) this wave's K steps and the weight fragments of its first D (MFMA-fragment order,
  // ConvArgs::wgt_f: one A fragment = one contiguous 1 KiB (16-bit) / 2 KiB (fp32) run)
  const int ns3 = nck * 9, ns = ns3 + rck;
  const int nj = wv < ns ? (ns - wv + NW - 1) / NW : 0;
  const int s_last = wv + NW * max(nj - 1, 0);
  const int cb0 = n0 / 16;
  const T* wbase = (const T*)a.wgt_f + (size_t)lane * 8;
  const T* rbase = (const T*)a.res_wgt_f + (size_t)lane * 8;
  auto wfrag = [&](int s, int fc) -> Frag<T> {
    const T* p = s < ns3 ? wbase + ((size_t)(cb0 + fc) * ns3 + s) * 512
                         : rbase + ((size_t)(cb0 + fc) * rck + (s - ns3)) * 512;
    return load_frag<T>((const char*)p);
  };
  Frag<T> wa[D][FC];
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int fc = 0; fc < FC; ++fc) wa[d][fc] = SDDM_DEEP_DBG(32) ? Frag<T>{} : wfrag(min(wv + NW * d, s_last), fc);
  DS_W(a);
  // (c) identity residual of this thread's epilogue pixels (4 channels each, clamped: unconditional)
  f32x4 idr[EIT];
  {
    const T* rsrc = (const T*)a.res_src + (size_t)b * img_out * gCout + n0 + ec4;
#pragma unroll
    for (int it = 0; it < EIT; ++it) {
      const int p = min(it * PPI + tid / TPP, npv - 1), py = p / gTW, px = p - py * gTW;
      const T* rp = ident ? rsrc + ((y0 + py) * gWo + (x0 + px)) * gCout : (const T*)g_deep_zero;
      idr[it] = load4<T>(rp);                            // unconditional (zero page without residual)
    }
  }
  // (d) the input halo by LDS-DMA, last: its loops issue a block-dependent number of DMAs, and
  // a register load issued after them would be waited for with vmcnt(0) (the compiler cannot
  // count them); everything above is straight-line, so its waits stay exact.  Per 64-pixel chunk
  // r: this lane's halo pixel -> source pixel (computed once, reused for every plane), then one
  // DMA per plane of this wave; bit r of `inb`: the pixel lies inside the image
  auto dma = [&](const char* src, char* dst) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
  };
  unsigned inb = 0;
  {
    const float rHC = 1.0f / (float)HC;
    for (int r = 0; r < geo.NCH; ++r) {                  // block-uniform
      const int hp = r * 64 + lane, hy = fdivi(hp, rHC), hx = hp - hy * HC;
      int iy, ix;
      bool ok;
      if (S2) {
        iy = 2 * y0 - 1 + hy; ix = 2 * x0 - 1 + hx;
        ok = iy >= 0 && iy < gHi && ix >= 0 && ix < gWi;
      } else {
        iy = y0 - 1 + hy; ix = x0 - 1 + hx;
        ok = iy >= 0 && iy < gHo && ix >= 0 && ix < gWo;
        if (gUp) { iy >>= 1; ix >>= 1; }
      }
      ok = ok && hp < geo.HP;
      inb |= ok ? 1u << r : 0u;
      const unsigned pix = ok ? (unsigned)(iy * gWi + ix) : 0u;
      const char* pa = ok ? srcA + pix * (unsigned)(gCA * ES) : zero;
      const char* pb = ok ? srcB + pix * (unsigned)(gCB * ES) - plA * 16 : zero;
      const unsigned step = ok ? 16u : 0u;               // the zero page for every plane outside
      char* dl = smem + r * 1024;
      for (int q = wv; q < npl; q += NW)                 // wave-uniform planes
        if (!SDDM_DEEP_DBG(4)) dma((q < plA ? pa : pb) + q * step, dl + q * PLB);
    }
  }
  // (e) the res_conv input at the output pixels (1x1, raw concat)
  if (rck) {
    const char* rawA = (const char*)a.rawA + (size_t)b * img_out * gRCA * ES;
    const char* rawB = (const char*)(gRCB ? a.rawB : a.rawA) + (size_t)b * img_out * gRCB * ES;
    for (int r = 0; r < geo.NCR; ++r) {
      const int p = r * 64 + lane, py = p / gTW, px = p - py * gTW;
      const int pix = p < npv ? (y0 + py) * gWo + (x0 + px) : -1;
      const unsigned oa = (unsigned)pix * (unsigned)(gRCA * ES), ob = (unsigned)pix * (unsigned)(gRCB * ES);
      for (int q = wv; q < nplr; q += NW) {
        const char* src = q < plRA ? rawA + oa + q * 16 : rawB + ob + (q - plRA) * 16;
        dma(pix >= 0 ? src : zero, smem + res_off + q * PLR + r * 1024);
      }
    }
  }
  DS_STG(a);
  // (f) bias + noise embedding of this thread's 4 epilogue channels (after the DMAs: the row
  // depends on the step counter's scalar round trip)
  float bb[4], sshift;
  {
    const float* trow = a.temb ? a.temb + (size_t)t_now * a.temb_ld : a.bias;
#pragma unroll
    for (int i = 0; i < 4; ++i) {                        // unconditional loads (no wait at a join)
      const float bv = a.bias[n0 + ec4 + i], tv = trow[n0 + ec4 + i];
      bb[i] = bv + (a.temb ? tv : 0.f);
    }
    const int cs = n0 + (tid & (NB - 1));                // statistics shift of channel n0 + tid (tid < NB)
    const float sbv = a.bias[cs], stv = trow[cs];
    sshift = sbv + (a.temb ? stv : 0.f);
  }
  DS_ISSUED(a);

  // ---------------- 2. GroupNorm finalize ----------------
  if (gn) gl.finish(gf, b, gCA, gCB, gsc, gsc + Cin);
  dma_sync();                                            // every wave's DMAs landed, scale / shift visible
  DS_LANDED(a);

  // ---------------- 3. GroupNorm + SiLU in place (zero padding stays zero) ----------------
  if (gn) {
    // two planes per pass (the second clamped to the first when the wave has an odd count), so
    // the LDS round trips of one overlap the transcendentals of the other
    for (int q0 = wv; q0 < npl; q0 += 2 * NW) {
      const bool two = q0 + NW < npl;                    // wave-uniform
      const int q1 = two ? q0 + NW : q0;
      float s0[VE], h0[VE], s1[VE], h1[VE];
#pragma unroll
      for (int j = 0; j < VE; j += 4) {                  // wave-uniform (broadcast) reads
        const f32x4 x0 = *(const f32x4*)(gsc + q0 * VE + j), y0 = *(const f32x4*)(gsc + Cin + q0 * VE + j);
        const f32x4 x1 = *(const f32x4*)(gsc + q1 * VE + j), y1 = *(const f32x4*)(gsc + Cin + q1 * VE + j);
#pragma unroll
        for (int i = 0; i < 4; ++i) { s0[j + i] = x0[i]; h0[j + i] = y0[i]; s1[j + i] = x1[i]; h1[j + i] = y1[i]; }
      }
      for (int r = 0; r < geo.NCH; ++r) {
        if ((inb >> r) & 1u) {
          f32x4* p0 = (f32x4*)(smem + q0 * PLB + r * 1024 + lane * 16);
          f32x4* p1 = (f32x4*)(smem + q1 * PLB + r * 1024 + lane * 16);
          const f32x4 v0 = *p0, v1 = *p1;
          const f32x4 o0 = transform_regs<T>(v0, s0, h0), o1 = transform_regs<T>(v1, s1, h1);
          *p0 = o0;
          if (two) *p1 = o1;
        }
      }
    }
    lds_sync();
  }
  DS_XFORM(a);

  // ---------------- 4. this wave's K steps ----------------
  int pix_off[FP];
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    int p = fp * 16 + (lane & 15);
    if (p >= npv) p = 0;
    const int py = p / gTW, px = p - py * gTW;
    pix_off[fp] = S2 ? ((2 * py) * HC + 2 * px) * 16 : (py * HC + px) * 16;
  }
  f32x4 acc[FP][FC];
#pragma unroll
  for (int i = 0; i < FP; ++i)
#pragma unroll
    for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nj; j0 += D) {
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
  DS_KLOOP(a);

  // ---------------- 5. reduce the partial tiles: red[slot][MT][NBP] ----------------
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

  float sn = 0.f, s1[4], s2[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { s1[i] = 0.f; s2[i] = 0.f; }
  T* out = (T*)a.out + (size_t)b * img_out * gCout + n0 + ec4;
#pragma unroll
  for (int it = 0; it < EIT; ++it) {
    const int p = it * PPI + tid / TPP;
    if (p < npv) {
      const int py = p / gTW, px = p - py * gTW;
      f32x4 s = *(const f32x4*)(red + p * NBP + ec4);
#pragma unroll
      for (int w = 1; w < SLOTS; ++w) s += *(const f32x4*)(red + (w * MT + p) * NBP + ec4);
      float d[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) d[i] = s[i] + idr[it][i];
      store4<T>(out + ((y0 + py) * gWo + (x0 + px)) * gCout, d[0] + bb[0], d[1] + bb[1], d[2] + bb[2], d[3] + bb[3]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {                    // sums about the shift bb (the same for
        s1[i] += d[i];                                 // every thread of a channel: they add)
        s2[i] += d[i] * d[i];
      }
      sn += 1.f;
    }
  }
  DS_STORED(a);
  if (a.stats) {
    // the lanes of a wave holding the same 4 channels (64 / TPP of them, TPP apart) add by DPP
    // row rotations and two cross-row swizzles, then the NW wave sums through LDS, summed by one
    // thread per channel in wave order
    auto wred = [](float x) {
      if constexpr (TPP == 4) x += dpp_f32<0x124>(x);   // row_ror:4
      if constexpr (TPP <= 8) x += dpp_f32<0x128>(x);   // row_ror:8
      x += __shfl_xor(x, 16);
      return x + __shfl_xor(x, 32);
    };
    const float tn = wred(sn);
    float t1[4], t2[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { t1[i] = wred(s1[i]); t2[i] = wred(s2[i]); }
    lds_sync();                                        // red reads done
    float* xs = red;                                   // [NW][NB channels][3]
    if (lane < TPP)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float* e = xs + (wv * NB + ec4 + i) * 3;
        e[0] = tn; e[1] = t1[i]; e[2] = t2[i];
      }
    lds_sync();
    if (tid < NB) {
      float n = 0.f, u1 = 0.f, u2 = 0.f;
#pragma unroll
      for (int r = 0; r < NW; ++r) {
        const float* e = xs + (r * NB + tid) * 3;
        n += e[0]; u1 += e[1]; u2 += e[2];
      }
      float* dst = a.stats + (((size_t)b * gNT + tile) * gCout + n0 + tid) * 2;
      dst[0] = (sshift + u1 / n) * n;
      dst[1] = fmaxf(u2 - u1 * u1 / n, 0.f);
    }
  }
  DS_STATS(a);
  SDDM_STAMP(a, 7);
}

// weight-ring depth for a wave's K steps: the whole K when it fits in the register budget
template <typename T, int MT, int NW>
static int deep_ring(int steps_per_wave) {
  if (sizeof(T) == 4 || NW == 4) return 8 / (int)(sizeof(T) == 4 ? 2 : 1);
  if (steps_per_wave <= 8 || MT >= 128) return 8;
  return 12;
}

template <typename T, bool S2, int MT, int NW, int NB, int SH = 0>
static hipError_t deep_go(const ConvArgs& a, int B, hipStream_t s, size_t* lo) {
  const int Cin = a.CA + a.CB, RC = a.res_mode == 2 ? a.RCA + a.RCB : 0;
  const int nck = Cin / 32, rck = RC / 32;
  const DeepGeo geo = deep_geo(S2, a.TR, a.TW, MT);
  const DeepLds lay = deep_layout<T, MT, NW, NB>(geo, Cin, RC);
  const bool fits = geo.NCH <= kDeepMaxChunks && geo.NCR <= 2;
  if (lo) {
    *lo = fits ? (size_t)lay.total : (size_t)1 << 40;
    return hipSuccess;
  }
  if (!fits || a.TR * a.TW > MT || a.Cout % NB || Cin % 32 || Cin > 1000 || RC % 32 || a.CA % 32)
    return hipErrorInvalidValue;
  if (lay.total > kLdsBytes) return hipErrorInvalidValue;
  const dim3 grid = xcd_grid(a.n_tiles, B, a.Cout / NB), blk(64 * NW);
  const int D = deep_ring<T, MT, NW>((nck * 9 + rck + NW - 1) / NW);
#define SDDM_RING(DV)                                                                         \
  if (D == DV) {                                                                              \
    hipLaunchKernelGGL((conv_deep_kernel<T, S2, MT, NW, DV, NB, SH>), grid, blk, lay.total, s, a); \
    return hipGetLastError();                                                                 \
  }
  if constexpr (NB == 64) {                               // 4 fragments per K step: a 4-step ring
    if constexpr (sizeof(T) == 4) {
      return hipErrorInvalidValue;                        // (16-bit only)
    } else {
      hipLaunchKernelGGL((conv_deep_kernel<T, S2, MT, NW, 4, NB, SH>), grid, blk, lay.total, s, a);
      return hipGetLastError();
    }
  } else if constexpr (SH > 0) {                          // one ring depth per specialised shape
    constexpr ConvShape c = kDeepShapes[SH];
    constexpr int spw = (((c.CA + c.CB) / 32) * 9 + (c.res == 2 ? (c.RCA + c.RCB) / 32 : 0) + NW - 1) / NW;
    constexpr int DS = (NW == 4 || MT >= 128 || spw <= 8) ? 8 : 12;
    SDDM_RING(DS)
  } else if constexpr (sizeof(T) == 4) {
    SDDM_RING(4)
  } else if constexpr (NW == 4 || MT >= 128) {
    SDDM_RING(8)
  } else {
    SDDM_RING(8) SDDM_RING(12)
  }
#undef SDDM_RING
  return hipErrorInvalidValue;
}

// the specialised shapes SH = 1 .. kNDeepShapes-1 (16-bit storage only) matching the launch
template <typename T, int SH>
static bool deep_shape_go(int mt, int nw, int nb, bool s2, const ConvArgs& a, int B, hipStream_t s, hipError_t& e) {
  if constexpr (SH >= kNDeepShapes || sizeof(T) == 4) {
    return false;
  } else if constexpr (!shape_for_type<T>(kDeepShapes[SH])) {
    return deep_shape_go<T, SH + 1>(mt, nw, nb, s2, a, B, s, e);
  } else {
    constexpr ConvShape c = kDeepShapes[SH];
    if (c.cfg == mt && c.nw == nw && c.nb == nb && conv_shape_geo_matches(c, s2, a)) {
      e = deep_go<T, c.s2 != 0, c.cfg, c.nw, c.nb, SH>(a, B, s, nullptr);
      return true;
    }
    return deep_shape_go<T, SH + 1>(mt, nw, nb, s2, a, B, s, e);
  }
}

// nb: output channels per block (32; 16 for twice the blocks with half the weight bytes each; 64
// for half the blocks, each transforming its input halo once for twice the output channels)
template <typename T>
static hipError_t deep_dispatch(int mt, int nw, int nb, bool s2, const ConvArgs& a, int B, hipStream_t s, size_t* lo) {
  static const bool generic = std::getenv("SDDM_NO_DEEP_SHAPES") != nullptr;   // A/B runs
  hipError_t e;
  if (!lo && !generic && deep_shape_go<T, 1>(mt, nw, nb, s2, a, B, s, e)) return e;
#define SDDM_DEEP(S2V, MTV, NWV, NBV) \
  if (s2 == S2V && mt == MTV && nw == NWV && nb == NBV) return deep_go<T, S2V, MTV, NWV, NBV>(a, B, s, lo);
  SDDM_DEEP(false, 32, 4, 32) SDDM_DEEP(false, 64, 4, 32) SDDM_DEEP(false, 128, 4, 32)
  SDDM_DEEP(true, 32, 4, 32) SDDM_DEEP(true, 64, 4, 32) SDDM_DEEP(true, 128, 4, 32)
  SDDM_DEEP(false, 32, 8, 32) SDDM_DEEP(false, 64, 8, 32) SDDM_DEEP(false, 128, 8, 32)
  SDDM_DEEP(true, 32, 8, 32) SDDM_DEEP(true, 64, 8, 32) SDDM_DEEP(true, 128, 8, 32)
  SDDM_DEEP(false, 16, 4, 16) SDDM_DEEP(false, 32, 4, 16) SDDM_DEEP(false, 64, 4, 16) SDDM_DEEP(false, 128, 4, 16)
  SDDM_DEEP(true, 16, 4, 16) SDDM_DEEP(true, 32, 4, 16) SDDM_DEEP(true, 64, 4, 16)
  SDDM_DEEP(false, 32, 8, 16) SDDM_DEEP(false, 64, 8, 16) SDDM_DEEP(false, 128, 8, 16)
  // 64-channel blocks (16-bit): a tile's halo transformed by half as many channel blocks (round 6)
  SDDM_DEEP(false, 32, 4, 64) SDDM_DEEP(false, 64, 4, 64) SDDM_DEEP(false, 32, 8, 64)
  SDDM_DEEP(true, 32, 4, 64) SDDM_DEEP(true, 64, 4, 64)
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

int conv_deep_ring_depth(int dtype, int mt, int nw, int ksteps, int nb) {
  const int spw = (ksteps + nw - 1) / nw;
  if (dtype == DT_F32 || nb == 64) return 4;
  if (nw == 4 || mt >= 128) return 8;
  return deep_ring<bf16_t, 64, 8>(spw);
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
