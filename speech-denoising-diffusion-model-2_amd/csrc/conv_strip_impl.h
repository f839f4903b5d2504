// Row-streaming ("line buffer") 3x3 convolution (kernel template; instantiated per storage type
// by conv_strip_bf16.hip / conv_strip_f16.hip / conv_strip_f32.hip, dispatched by conv_strip.hip) for the wide UNet levels (segment width W = 128
// and 64: UNetModified2 levels 0-1, where >60 % of the FLOPs live).
//
// One block owns image b, output channels [n0, n0 + 16*FC) and a strip of SR output rows.  It
// keeps in LDS
//   * the weight slab of its channel tile (loaded once per strip, not once per tile), and
//   * a ring of R = 2*TR + 2 transformed input rows (GroupNorm + SiLU applied once per element,
//     zero halo columns, nearest-2x upsample / channel concat resolved while loading),
// and walks the strip TR = MPI / W output rows at a time (MPI = 128 or 256 pixels, one wave per
// 32 pixels = 2 MFMA column fragments; with MPI = 256 each SIMD runs two waves, so one wave's
// GN+SiLU staging overlaps the other's MFMAs).  While the MFMAs of iteration i run on rows [y-1, y+TR] of the ring, each thread
// already holds in registers the raw input of rows [y+TR+1, y+2TR] (issued before the MFMAs) and
// writes them transformed into the free ring slots afterwards: one barrier per iteration.
//
// LDS images are plane-major (a plane = one 16-byte channel unit of every pixel / output channel,
// plane stride = 0 mod 256 B): the 16 lanes of an MFMA operand read 16 consecutive 16-byte slots
// and the ds_read_b128 lane groups never collide; staging writes go 8 consecutive pixels per
// 8-lane group (conflict free) while the 64 lanes of a wave read 64/UPP whole pixels (coalesced).
// Geometry (W, Cin) is compile-time so no integer division runs per element.
// The epilogue adds bias, the noise-embedding projection and the residual (identity, or the
// ResnetBlock 1x1 res_conv as extra MFMAs on raw input fragments loaded straight to registers),
// stores 4 channels per lane, and accumulates GroupNorm statistics of the fp32 values in
// registers (per-lane shifted sums, merged with Chan's formula at the end of the strip).
//
// Memory pipelining: the rows of row group j + 2 are issued at the top of iteration j into one of
// two register sets (period-2 rotation, the loop unrolled by two) and committed at the end of
// iteration j + 1, and the residual inputs (identity tile or res_conv fragments, RES = 1 / 2, a
// template parameter so no load sits under a runtime branch) one iteration ahead.  Every body is
// straight-line code, so the compiler's memory-counter waits are exact, and the iteration barrier
// orders LDS only: no iteration waits for the loads it issued.
#pragma once
#include <type_traits>

// timing-ablation builds only (tools/gpu_ablate.sh): 16 every tap reads the same weight fragment,
// 256 every tap reads the same input fragment (results are garbage)
#ifndef SDDM_ABL_STRIP
#define SDDM_ABL_STRIP 0
#endif
#ifndef SDDM_STRIP_WLD
#define SDDM_STRIP_WLD 1   // 0: weight slabs by LDS-DMA only (A/B builds)
#endif
#ifndef SDDM_STRIP_WREG
#define SDDM_STRIP_WREG 1   // 0: weight fragments re-read from LDS every iteration (A/B builds)
#endif

#include "conv_common.h"
#include "conv_tile_cfg.h"
#include "kernels.h"

namespace sddm {

// strip kernel shapes (conv_tile_cfg.h ConvShape; cfg = output channels per block, TR = nb =
// strip rows, TW = W, nw = pixels per iteration): UNetModified2 config_unet.json at 16448 samples
// with the kernels of configs/conv_tuning.json
static constexpr ConvShape kStripShapes[] = {
    {-1, 0, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},   // generic (fields unused)
    {32, 0, 16, 128, 256, 128, 32, 0, 32, 0, 0, 0, 1, 0, 256, 16},      // downs.1.block1
    {32, 0, 16, 128, 256, 128, 32, 0, 32, 0, 0, 1, 1, 0, 256, 16},      // downs.1.block2
    {64, 0, 8, 64, 128, 64, 32, 0, 64, 0, 0, 0, 1, 0, 256, 8},          // downs.3.block1
    {32, 0, 16, 64, 128, 64, 64, 0, 64, 32, 0, 2, 1, 0, 256, 16},       // downs.3.block2
    {32, 0, 16, 64, 128, 64, 64, 0, 64, 0, 0, 0, 0, 1, 256, 16},        // ups.10 (Upsample)
    {32, 0, 8, 64, 128, 64, 32, 0, 32, 64, 64, 2, 1, 0, 256, 8},        // ups.11.block2
    {32, 0, 8, 64, 128, 64, 32, 32, 32, 0, 0, 0, 1, 0, 256, 8},         // ups.12.block1
    {32, 0, 8, 64, 128, 64, 32, 0, 32, 32, 32, 2, 1, 0, 256, 8},        // ups.12.block2
    {32, 0, 16, 128, 256, 128, 32, 0, 32, 0, 0, 0, 0, 1, 256, 16},      // ups.13 (Upsample)
    {32, 0, 16, 128, 256, 128, 32, 32, 32, 0, 0, 0, 1, 0, 256, 16},     // ups.14.block1
    {32, 0, 16, 128, 256, 128, 32, 0, 32, 32, 32, 2, 1, 0, 256, 16},    // ups.14.block2
    // BASELINE config #5 per GPU (32832 samples, 64-row lanes, fp16) with its measured table
    {32, 0, 64, 128, 512, 128, 32, 0, 32, 0, 0, 0, 1, 0, 256, 64, 1},   // c5:downs.1.block1
    {32, 0, 64, 128, 512, 128, 32, 0, 32, 0, 0, 1, 1, 0, 256, 64, 1},   // c5:downs.1.block2
    {64, 0, 64, 64, 256, 64, 32, 0, 64, 0, 0, 0, 1, 0, 256, 64, 1},     // c5:downs.3.block1
    {32, 0, 128, 64, 256, 64, 64, 0, 64, 32, 0, 2, 1, 0, 256, 128, 1},  // c5:downs.3.block2
    {32, 0, 128, 64, 256, 64, 64, 0, 64, 0, 0, 0, 0, 1, 256, 128, 1},   // c5:ups.10
    {32, 0, 64, 64, 256, 64, 32, 0, 32, 64, 64, 2, 1, 0, 256, 64, 1},   // c5:ups.11.block2
    {32, 0, 64, 64, 256, 64, 32, 32, 32, 0, 0, 0, 1, 0, 256, 64, 1},    // c5:ups.12.block1
    {32, 0, 64, 64, 256, 64, 32, 0, 32, 32, 32, 2, 1, 0, 256, 64, 1},   // c5:ups.12.block2
    {32, 0, 64, 128, 512, 128, 32, 0, 32, 0, 0, 0, 0, 1, 256, 64, 1},   // c5:ups.13
    {32, 0, 64, 128, 512, 128, 32, 32, 32, 0, 0, 0, 1, 0, 256, 64, 1},  // c5:ups.14.block1
    {32, 0, 64, 128, 512, 128, 32, 0, 32, 32, 32, 2, 1, 0, 256, 64, 1}, // c5:ups.14.block2
};
static constexpr int kNStripShapes = (int)(sizeof(kStripShapes) / sizeof(kStripShapes[0]));

__host__ inline bool strip_shape_matches(const ConvShape& c, int nblk, int mpi, int SR, const ConvArgs& a) {
  return c.cfg == nblk && c.nw == mpi && c.nb == SR && c.Ho == a.Ho && c.Wo == a.Wo && c.CA == a.CA && c.CB == a.CB &&
         c.Cout == a.Cout && c.RCA == a.RCA && c.RCB == a.RCB && c.res == a.res_mode &&
         c.gn == (a.gamma != nullptr ? 1 : 0) && c.up == (a.upsample ? 1 : 0) && a.n_tiles == c.Ho / SR &&
         a.Hi == (c.up ? c.Ho / 2 : c.Ho) && a.Wi == (c.up ? c.Wo / 2 : c.Wo);
}

template <typename T, int FC, int W, int CIN, int MPI, int RES, bool GN, int SH>
__global__ __launch_bounds__(MPI * 2) void conv_strip_kernel(ConvArgs a, int SR_) {
  // layer geometry: compile-time for a specialised shape (SH > 0), else the arguments
  constexpr ConvShape SC = kStripShapes[SH];
  constexpr bool CS = SH > 0;
  SDDM_SHAPE_GEO(SC, CS, false, a)
  const int SR = CS ? SC.nb : SR_;
  (void)gTR; (void)gTW; (void)gTX; (void)gRes; (void)gGN; (void)gWo;
  constexpr int NT = MPI * 2;                     // threads: one wave per 32 pixels of an iteration
  constexpr int NWV = NT / 64;
  constexpr int ES = (int)sizeof(T);
  constexpr int NBLK = 16 * FC, FP = 2;
  constexpr int TR = MPI / W, R = 2 * TR + 2;
  constexpr int UPP = CIN * ES / 16;              // 16-byte channel units (planes) per pixel
  constexpr int UPL = ES / 2;                     // units per lane group (8 channels)
  constexpr int VE = 16 / ES;
  constexpr int PL = ((W + 2) * 16 + 255) / 256 * 256;
  constexpr int SLOT = UPP * PL;
  constexpr int NCK = CIN / 32;
  constexpr int WPL = NBLK * 16;                  // weight plane stride
  constexpr int WPLANES = NCK * 9 * 4 * UPL;
  constexpr int PB = 64 / UPP;                    // pixels per 64-unit staging group
  constexpr int NU = TR * W * UPP;                // units of TR rows
  constexpr int UPT = NU / NT;                    // prefetch units per thread and row group
  constexpr int IU = ((TR + 2) * W * UPP + NT - 1) / NT;   // initial-row units per thread
  constexpr int RCKM = 4;                         // res_conv chunks held in registers (RC <= 128)
  static_assert(UPP >= 1 && UPP <= 64 && (64 % UPP) == 0, "channel units must divide a wave");
  static_assert(NU % NT == 0, "prefetch must split evenly");
  typedef T vec4 __attribute__((ext_vector_type(4)));
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  int strip, b, zb;
  xcd_block<SDDM_XCD_ZIN != 0>(gNT, gCout / NBLK, strip, b, zb);
  const int n0 = zb * NBLK;
  const int H = gHo;
  const int RC = gRCA + gRCB;
  const int rck = RES == 2 ? RC / 32 : 0;
  constexpr bool gn = GN;                         // GroupNorm + SiLU on the input (a Block conv)

  char* ring = smem;                              // [R][UPP planes][PL]
  char* wl = ring + R * SLOT;                     // [WPLANES][NBLK][16 B]
  char* rw = wl + WPLANES * WPL;                  // [RC*ES/16 planes][NBLK][16 B]
  const int RPLANES = rck * 32 * ES / 16;
  float* gsc = (float*)(rw + RPLANES * WPL);      // [2][CIN]
  float* red = gsc + 2 * CIN;                     // [NWV waves][NBLK][3]

  const int y0 = strip * SR;
  const int iters = SR / TR;                      // even (checked by the launcher)
  SDDM_STAMP(a, 0);
  // ---------------- prologue: every independent load issued before anything waits ----------------
  GNLoad gl;
  const GNFuse gf{a.gstA, a.gtilesA, a.gntileA, a.gstB, a.gtilesB, a.gntileB, a.gamma, a.beta, a.groups, a.eps};
  gl.issue(gf, b, gCA, gCB, gn, a.bias);
  // initial ring rows y0-1 .. y0+TR (raw), clamped addresses, zero rows outside the image later
  const T* srcAb = (const T*)a.srcA + (size_t)b * gHi * gWi * gCA;
  const T* srcBb = gCB ? (const T*)a.srcB + (size_t)b * gHi * gWi * gCB : srcAb;
  f32x4 ini[IU];
#pragma unroll
  for (int k = 0; k < IU; ++k) {
    const int u = min(tid + k * NT, (TR + 2) * W * UPP - 1);
    const int grp = u >> 6, j = u & 63;
    const int pix = grp * PB + (j % PB), q = j / PB, r = pix / W, x = pix % W;
    const int ry = min(max(y0 - 1 + r, 0), H - 1);
    const int sy = gUp ? ry >> 1 : ry, sx = gUp ? x >> 1 : x;
    const int c0 = q * VE;
    const bool fa = c0 < gCA;
    ini[k] = *(const f32x4*)((fa ? srcAb : srcBb) + ((size_t)sy * gWi + sx) * (fa ? gCA : gCB) + (fa ? c0 : c0 - gCA));
  }
  // weight slabs: through registers (WLD: WU / RU fixed 16-byte units per thread, clamped loads,
  // written to LDS after the initial ring rows; a global load + ds_write per unit issues cheaper
  // than an LDS-DMA, strips -4..-6 us per step, bench +1 %), or, for slabs of more
  // than 12 units per thread (Cin = 128: too many VGPRs), by LDS-DMA.  Unit u lands at byte 16 u,
  // co fastest.  16-bit weights come from the chunk-major image ConvArgs::wgt_t
  // ([Cin/32][9][4][Cout][8]): the NBLK channels of one plane are one contiguous run, so a
  // wave-instruction reads 1 KiB of consecutive bytes.  From the per-channel image (fp32) each
  // lane reads another channel's row.
  constexpr int WUN = NBLK * WPLANES, WU = (WUN + NT - 1) / NT;
  constexpr bool WLD = SDDM_STRIP_WLD && WU <= 12;
  constexpr int RUN_MAX = RES == 2 ? NBLK * RCKM * 4 * UPL : 0, RU = (RUN_MAX + NT - 1) / NT;
  const int RUN = NBLK * RPLANES;
  f32x4 wst[WLD ? WU : 1], rst[WLD && RU > 0 ? RU : 1];
  if constexpr (WLD) {
#pragma unroll
    for (int i = 0; i < WU; ++i) {
      const int u0 = tid + i * NT, u = u0 < WUN ? u0 : 0;
      const int co = u % NBLK, pl = u / NBLK;                 // pl = (ck*9 + tap)*4*UPL + unit
      const char* src;
      if constexpr (ES == 2) {
        src = (const char*)a.wgt_t + ((size_t)pl * gCout + n0 + co) * 16;
      } else {
        const int ck = pl / (9 * 4 * UPL), rem = pl - ck * 9 * 4 * UPL, tap = rem / (4 * UPL), un = rem - tap * 4 * UPL;
        src = (const char*)a.wgt + ((((size_t)(n0 + co) * NCK + ck) * 9 + tap) * 32) * ES + un * 16;
      }
      wst[i] = *(const f32x4*)src;
    }
    if constexpr (RES == 2) {
#pragma unroll
      for (int i = 0; i < RU; ++i) {
        const int u0 = tid + i * NT, u = u0 < RUN ? u0 : 0;
        const int co = u % NBLK, pl = u / NBLK;
        const char* src = ES == 2 ? (const char*)a.res_wgt_t + ((size_t)pl * gCout + n0 + co) * 16
                                  : (const char*)a.res_wgt + ((size_t)(n0 + co) * RC) * ES + pl * 16;
        rst[i] = *(const f32x4*)src;
      }
    }
  } else {
    // LDS-DMA: every wave-instruction fills 1 KiB of consecutive LDS, no VGPRs, no wait until the
    // first barrier; NBLK * WPLANES and NBLK * RPLANES are multiples of 64: whole waves, no tail
    for (int u0 = wave * 64; u0 < NBLK * WPLANES; u0 += NT) {
      const int u = u0 + lane;
      const int co = u % NBLK, pl = u / NBLK;                 // pl = (ck*9 + tap)*4*UPL + unit
      const char* src;
      if constexpr (ES == 2) {
        src = (const char*)a.wgt_t + ((size_t)pl * gCout + n0 + co) * 16;
      } else {
        const int ck = pl / (9 * 4 * UPL), rem = pl - ck * 9 * 4 * UPL, tap = rem / (4 * UPL), un = rem - tap * 4 * UPL;
        src = (const char*)a.wgt + ((((size_t)(n0 + co) * NCK + ck) * 9 + tap) * 32) * ES + un * 16;
      }
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                       (__attribute__((address_space(3))) void*)(wl + u0 * 16), 16, 0, 0);
    }
    if constexpr (RES == 2) {
      for (int u0 = wave * 64; u0 < NBLK * RPLANES; u0 += NT) {
        const int u = u0 + lane;
        const int co = u % NBLK, pl = u / NBLK;
        const char* src = ES == 2 ? (const char*)a.res_wgt_t + ((size_t)pl * gCout + n0 + co) * 16
                                  : (const char*)a.res_wgt + ((size_t)(n0 + co) * RC) * ES + pl * 16;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)(rw + u0 * 16), 16, 0, 0);
      }
    }
  }
  for (int u = tid; u < R * UPP * 2; u += NT) {           // zero halo columns
    const int side = u & 1, pl = u >> 1;
    *(f32x4*)(ring + pl * PL + (side ? (W + 1) : 0) * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (gn) gl.finish(gf, b, gCA, gCB, gsc, gsc + CIN);
  __syncthreads();                                         // gsc ready
  // bias + noise embedding of this lane's epilogue channels (Cout % NBLK == 0: no clamping)
  const int t_now = a.t_dev ? *a.t_dev : 0;
  const float* trow = a.temb ? a.temb + (size_t)(a.temb_per_b ? b : t_now) * a.temb_ld : a.bias;
  float badd[FC][4];
#pragma unroll
  for (int fc = 0; fc < FC; ++fc)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = n0 + fc * 16 + 4 * g + i;
      const float bv = a.bias[co], tv = trow[co];
      badd[fc][i] = bv + (a.temb ? tv : 0.f);
    }
  // the statistics shift of channel n0 + tid (threads tid < NBLK write the tile statistics):
  // loaded here so the end of the strip does not wait a memory round trip for it
  float sshift;
  {
    const int cs = n0 + (tid % NBLK);
    const float bv = a.bias[cs], tv = trow[cs];
    sshift = bv + (a.temb ? tv : 0.f);
  }
  const int base = ((y0 - 1) % R + R) % R;                 // ring slot of row y0 - 1
#pragma unroll
  for (int k = 0; k < IU; ++k) {
    const int u = tid + k * NT;
    if (u >= (TR + 2) * W * UPP) break;
    const int grp = u >> 6, j = u & 63;
    const int pix = grp * PB + (j % PB), q = j / PB, r = pix / W, x = pix % W;
    const int ry = y0 - 1 + r;
    f32x4 v = ini[k];
    if (ry < 0 || ry >= H) v = f32x4{0.f, 0.f, 0.f, 0.f};
    else if (gn) v = transform_fast<T>(v, gsc + q * VE, gsc + CIN + q * VE);
    *(f32x4*)(ring + ((base + r) % R) * SLOT + q * PL + (x + 1) * 16) = v;
  }

  if constexpr (WLD) {
#pragma unroll
    for (int i = 0; i < WU; ++i)
      if (tid + i * NT < WUN) *(f32x4*)(wl + (tid + i * NT) * 16) = wst[i];
    if constexpr (RES == 2) {
#pragma unroll
      for (int i = 0; i < RU; ++i)
        if (tid + i * NT < RUN) *(f32x4*)(rw + (tid + i * NT) * 16) = rst[i];
    }
  }

  // a 16-pixel column fragment never crosses a row (W % 16 == 0), so its row is wave-uniform: the
  // per-iteration ring-slot and row arithmetic below is scalar
  static_assert(W % 32 == 0, "a wave's 32 pixels must not cross rows");
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  int prow[FP], pcol[FP];
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    // (W % 32 == 0: both fragments of a wave share its row, fragment 1 sits 16 pixels right)
    prow[fp] = (wave_u * 32) / W;
    pcol[fp] = (wave_u * 32) % W + fp * 16 + (lane & 15);
  }
  // row-group prefetch geometry of this thread's units (the same every iteration)
  // (all per-iteration address math below is 32-bit with 24-bit multiplies: full-rate VALU)
  // (global addresses below are a base plus an unsigned 32-bit byte offset: no sign extensions and,
  // where the base is uniform, the scalar-base addressing form)
  int pr[UPT], loff[UPT], cq[UPT];              // row in group, LDS offset, channel
  const char* rsrc_[UPT];                       // this unit's column / channel in row 0 of its source
  unsigned rstr[UPT];                           // its source's row stride in bytes
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    const int u = tid + k * NT, grp = u >> 6, j = u & 63;
    const int pix = grp * PB + (j % PB);
    const int q = j / PB, x = pix % W;
    pr[k] = pix / W;
    loff[k] = q * PL + (x + 1) * 16;
    cq[k] = q * VE;
    const int c0 = q * VE;
    const int sx = gUp ? (x >> 1) : x;
    const bool fa = c0 < gCA;
    rsrc_[k] = fa ? (const char*)(srcAb + sx * gCA + c0) : (const char*)(srcBb + sx * gCB + (c0 - gCA));
    rstr[k] = (unsigned)(gWi * (fa ? gCA : gCB) * ES);
  }
  // rows of row group j (clamped: the groups past the strip end load valid rows nobody reads)
  auto issue_rows = [&](f32x4 (&dst)[UPT], int j) {
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      const int ry = min(y0 + j * TR + 1 + pr[k], H - 1);
      const int sy = gUp ? (ry >> 1) : ry;
      dst[k] = *(const f32x4*)(rsrc_[k] + (unsigned)__umul24((unsigned)sy, rstr[k]));
    }
  };
  // ring slots of row group j (group iters, past the strip, lands in slots nobody reads again)
  // unit k of row group j, transformed (branch-free: rows past the image are zeroed by a select,
  // so the transform stays in the iteration's basic block, interleaved with the MFMAs)
  auto xform_unit = [&](const f32x4 (&src)[UPT], int j, int k) {
    const int ry = y0 + j * TR + 1 + pr[k];
    f32x4 v = src[k];
    if constexpr (GN) v = transform_lds<T>(v, gsc + cq[k], gsc + CIN + cq[k]);
    return ry >= H ? f32x4{0.f, 0.f, 0.f, 0.f} : v;
  };
  auto store_rows = [&](const f32x4 (&tv)[UPT], int j) {
    const int sb = (base + j * TR + 2) % R;             // uniform
#pragma unroll
    for (int k = 0; k < UPT; ++k) {
      int sl = sb + pr[k];
      sl = sl >= R ? sl - R : sl;
      *(f32x4*)(ring + (int)__umul24(sl, SLOT) + loff[k]) = tv[k];
    }
  };
  T* outb = (T*)a.out + (size_t)b * H * W * gCout;
  // residual inputs of iteration it (issued one iteration ahead; rows clamped into the image)
  const T* resb = RES == 1 ? (const T*)a.res_src + (size_t)b * H * W * gCout : outb;
  auto issue_res1 = [&](vec4 (&dst)[FP][FC], int it) {
#pragma unroll
    for (int fp = 0; fp < FP; ++fp) {
      const int yy = min(y0 + it * TR, H - TR) + prow[fp];
      const unsigned po = (unsigned)(yy * W * gCout) + __umul24((unsigned)pcol[fp], (unsigned)gCout) + n0 + 4 * g;
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) dst[fp][fc] = *(const vec4*)((const char*)resb + (po * ES + fc * 16 * ES));
    }
  };
  const T* rawAb = RES == 2 ? (const T*)a.rawA + (size_t)b * H * W * gRCA : outb;
  const T* rawBb = (RES == 2 && gRCB) ? (const T*)a.rawB + (size_t)b * H * W * gRCB : rawAb;
  auto issue_res2 = [&](Frag<T> (&dst)[RCKM][FP], int it) {
#pragma unroll
    for (int ck = 0; ck < RCKM; ++ck)
#pragma unroll
      for (int fp = 0; fp < FP; ++fp) {
        const int yy = min(y0 + it * TR, H - TR) + prow[fp];
        const int c0 = min(ck, rck - 1) * 32 + g * 8;
        const int pix = yy * W + pcol[fp];
        const T* sp = c0 < gRCA ? rawAb + ((int)__umul24(pix, gRCA) + c0) : rawBb + ((int)__umul24(pix, gRCB) + (c0 - gRCA));
        dst[ck][fp] = load_frag<T>((const char*)sp);
      }
  };

  // per-lane sums of (value - badd) (shift = bias + embedding) as packed pairs matching the
  // accumulator register pairs: the epilogue is v_pk_add / v_pk_fma, no shuffles
  f32x2 s1[FC][2], s2[FC][2], bp[FC][2];
#pragma unroll
  for (int fc = 0; fc < FC; ++fc)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      s1[fc][h] = f32x2{0.f, 0.f};
      s2[fc][h] = f32x2{0.f, 0.f};
      bp[fc][h] = f32x2{badd[fc][2 * h], badd[fc][2 * h + 1]};
    }
  const char* abase = wl + g * UPL * WPL + (lane & 15) * 16;
  const char* rbase = rw + g * UPL * WPL + (lane & 15) * 16;

  // one iteration: loads of row group it+2 and the next residual inputs, MFMAs on the ring rows
  // of row group it, epilogue, ring refill with row group it+1 (issued one iteration earlier)
  f32x4 rowsA[UPT], rowsB[UPT];
  vec4 r1A[FP][FC], r1B[FP][FC];
  Frag<T> r2A[RCKM][FP], r2B[RCKM][FP];
  // LR / LX (compile-time): issue the rows of row group it + 2 / the residual inputs of iteration
  // it + 1 and refill the ring; the last two iterations of a strip issue no rows and the last
  // neither residual inputs nor a refill (the groups past the strip end were once loaded clamped
  // and never read: up to 2x the input bytes of the 2-iteration level-1 strips)
  // one input-channel chunk, two channel fragments, 16-bit storage, no res_conv: the 9 x FC weight
  // fragments stay in VGPRs for the whole strip (72 VGPRs) instead of being re-read from LDS by
  // every iteration (half the operand reads)
  constexpr bool WREG = SDDM_STRIP_WREG && ES == 2 && NCK == 1 && FC == 2 && RES != 2 && MPI == 256;
  Frag<T> wreg[WREG ? 9 : 1][FC];
  auto body = [&](auto LR, auto LX, int it, f32x4 (&nxt)[UPT], f32x4 (&fill)[UPT], vec4 (&r1cur)[FP][FC],
                  vec4 (&r1nxt)[FP][FC], Frag<T> (&r2cur)[RCKM][FP], Frag<T> (&r2nxt)[RCKM][FP]) {
    const int y = y0 + it * TR;
    const int s_it = (base + it * TR) % R;               // slot of row y - 1
#ifdef SDDM_STAMPS
    // timing ablations of the profiling build (SDDM_STAMPS_DBG): 4 no row loads, 64 no residual
    // loads, 8 no MFMAs, 2 no staging transform, 128 no output stores (results are garbage)
    const int dbg = a.dbg;
#else
    constexpr int dbg = 0;
#endif
    if constexpr (decltype(LR)::value) if (!(dbg & 4)) issue_rows(nxt, it + 2);
    if constexpr (RES == 1 && decltype(LX)::value) if (!(dbg & 64)) issue_res1(r1nxt, it + 1);
    if constexpr (RES == 2 && decltype(LX)::value) issue_res2(r2nxt, it + 1);
    // keep these loads at the top of the body: the scheduler would otherwise sink them below the
    // MFMAs (shorter live ranges) and halve the prefetch distance
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[FP][FC];
#pragma unroll
    for (int i = 0; i < FP; ++i)
#pragma unroll
      for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* bptr[FP][3];
#pragma unroll
    for (int fp = 0; fp < FP; ++fp)
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        int sl = s_it + prow[fp] + dy;                   // < 2R: one conditional wrap
        sl = sl >= R ? sl - R : sl;
        bptr[fp][dy] = ring + (sl * SLOT + (g * UPL * PL + pcol[fp] * 16));
      }
    // the ring refill of row group it + 1 (its rows were issued an iteration ago) is transformed
    // between the taps' MFMAs, unit k after tap k * 9 NCK / UPT, and stored after the epilogue
    f32x4 tv[UPT];
#pragma unroll
    for (int ck = 0; ck < NCK; ++ck) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3, dx = tap - 3 * dy;
        Frag<T> bf[FP];
#pragma unroll
        for (int fp = 0; fp < FP; ++fp)   // (SDDM_ABL_STRIP & 256: every tap reads tap 0's fragment)
          bf[fp] = load_planes<T>((SDDM_ABL_STRIP & 256) ? bptr[fp][0] : bptr[fp][dy] + ck * 4 * UPL * PL + dx * 16, PL);
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) {
          const Frag<T> af = WREG ? wreg[WREG ? tap : 0][fc]
                                  : load_planes<T>(abase + ((SDDM_ABL_STRIP & 16) ? 0 : (ck * 9 + tap) * 4 * UPL * WPL) + fc * 256, WPL);
#pragma unroll
          for (int fp = 0; fp < FP; ++fp)
            if (!(dbg & 8)) mfma_frag(acc[fp][fc], af, bf[fp]);
        }
#pragma unroll
        for (int k = 0; k < UPT; ++k)                      // (the last iteration refills nothing)
          if (decltype(LX)::value && ck * 9 + tap == k * 9 * NCK / UPT) tv[k] = (dbg & 2) ? fill[k] : xform_unit(fill, it + 1, k);
      }
    }
    if constexpr (RES == 2) {  // ResnetBlock.res_conv 1x1 on the raw block input (fragments prefetched)
#pragma unroll
      for (int ck = 0; ck < RCKM; ++ck) {
        if (ck >= rck) break;
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) {
          const Frag<T> af = load_planes<T>(rbase + ck * 4 * UPL * WPL + fc * 256, WPL);
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) mfma_frag(acc[fp][fc], af, r2cur[ck][fp]);
        }
      }
    }
    // ---- epilogue: bias + embedding + residual, store, statistics ----
#pragma unroll
    for (int fp = 0; fp < FP; ++fp) {
      const unsigned po = (unsigned)((y + prow[fp]) * W * gCout) + __umul24((unsigned)pcol[fp], (unsigned)gCout);
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) {
        const unsigned co = n0 + fc * 16 + 4 * g;
        // statistics of the fp32 values (before the storage rounding), about the shift badd
        f32x2 d0 = f32x2{acc[fp][fc][0], acc[fp][fc][1]}, d1 = f32x2{acc[fp][fc][2], acc[fp][fc][3]};
        if constexpr (RES == 1) {
          d0 += unpack2<T>(r1cur[fp][fc][0], r1cur[fp][fc][1]);
          d1 += unpack2<T>(r1cur[fp][fc][2], r1cur[fp][fc][3]);
        }
        if (!(dbg & 128)) store4p<T>((T*)((char*)outb + (po + co) * ES), d0 + bp[fc][0], d1 + bp[fc][1]);
        s1[fc][0] += d0;
        s1[fc][1] += d1;
        s2[fc][0] = __builtin_elementwise_fma(d0, d0, s2[fc][0]);
        s2[fc][1] = __builtin_elementwise_fma(d1, d1, s2[fc][1]);
      }
    }
    if constexpr (decltype(LX)::value) store_rows(tv, it + 1);
    lds_sync();                                          // LDS only: the prefetches stay in flight
  };
  issue_rows(rowsA, 1);
  if constexpr (RES == 1) issue_res1(r1A, 0);
  if constexpr (RES == 2) issue_res2(r2A, 0);
  // the weight DMA and the initial ring must have landed before the first MFMA; the NYOUNG loads
  // just issued stay in flight (a counted wait: everything older has completed)
  constexpr int NYOUNG = UPT + (RES == 1 ? FP * FC : 0) + (RES == 2 ? RCKM * FP : 0);
  static_assert(NYOUNG < 64, "vmcnt is a 6-bit counter");
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" :: "n"(NYOUNG) : "memory");
  if constexpr (WREG) {
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) wreg[tap][fc] = load_planes<T>(abase + tap * 4 * UPL * WPL + fc * 256, WPL);
  }
  SDDM_STAMP(a, 3);
  using yes = std::integral_constant<bool, true>;
  using no = std::integral_constant<bool, false>;
  for (int it = 0; it < iters - 2; it += 2) {            // period-2 rotation of the register sets
    body(yes{}, yes{}, it, rowsB, rowsA, r1A, r1B, r2A, r2B);
    body(yes{}, yes{}, it + 1, rowsA, rowsB, r1B, r1A, r2B, r2A);
  }
  body(no{}, yes{}, iters - 2, rowsB, rowsA, r1A, r1B, r2A, r2B);
  body(no{}, no{}, iters - 1, rowsA, rowsB, r1B, r1A, r2B, r2A);

  SDDM_STAMP(a, 4);
  // ---- GroupNorm statistics of the strip: lanes -> waves -> block ----
  // every lane of a channel sums about the same shift badd, so the sums add directly: the 16
  // pixel lanes of a DPP row (VALU adds), then the waves through LDS
  if (a.stats) {
    const float nl = (float)(FP * iters) * 16.f;
#pragma unroll
    for (int fc = 0; fc < FC; ++fc)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float t1 = row_sum16(s1[fc][i >> 1][i & 1]), t2 = row_sum16(s2[fc][i >> 1][i & 1]);
        if ((lane & 15) == 0) {
          float* rr = red + ((wave * NBLK) + fc * 16 + 4 * g + i) * 3;
          rr[0] = nl; rr[1] = t1; rr[2] = t2;
        }
      }
    lds_sync();
    if (tid < NBLK) {
      float n = 0.f, u1 = 0.f, u2 = 0.f;
      for (int w = 0; w < NWV; ++w) {
        const float* rr = red + (w * NBLK + tid) * 3;
        n += rr[0]; u1 += rr[1]; u2 += rr[2];
      }
      float* dst = a.stats + (((size_t)b * gNT + strip) * gCout + n0 + tid) * 2;
      dst[0] = (sshift + u1 / n) * n;
      dst[1] = fmaxf(u2 - u1 * u1 / n, 0.f);
    }
  }
  SDDM_STAMP(a, 6);
  SDDM_STAMP(a, 7);
}

template <typename T, int FC, int W, int CIN, int MPI>
static size_t strip_lds(const ConvArgs& a) {
  constexpr int ES = (int)sizeof(T), NBLK = 16 * FC, TR = MPI / W, R = 2 * TR + 2;
  constexpr int UPP = CIN * ES / 16, PL = ((W + 2) * 16 + 255) / 256 * 256;
  size_t n = (size_t)R * UPP * PL + (size_t)(CIN / 32) * 9 * 4 * (ES / 2) * NBLK * 16;
  if (a.res_mode == 2) n += (size_t)((a.RCA + a.RCB) * ES / 16) * NBLK * 16;
  n += (size_t)2 * CIN * 4 + (size_t)(MPI / 32) * NBLK * 3 * 4;
  return n;
}

template <typename T, int FC, int W, int CIN, int MPI, int SH = 0>
static hipError_t strip_go(const ConvArgs& a, int SR, int B, hipStream_t s, size_t* lo) {
  const size_t lds = strip_lds<T, FC, W, CIN, MPI>(a);
  if (lo) { *lo = lds; return hipSuccess; }
  constexpr int TR = MPI / W;
  if (lds > kLdsBytes || a.Ho % SR || SR % (2 * TR) || a.Cout % (16 * FC) || a.res_mode < 0 || a.res_mode > 2 ||
      (a.res_mode == 2 && (a.RCA + a.RCB) > 128))
    return hipErrorInvalidValue;
  if (a.n_tiles != a.Ho / SR) return hipErrorInvalidValue;
  if (sizeof(T) == 2 && (!a.wgt_t || (a.res_mode == 2 && !a.res_wgt_t))) return hipErrorInvalidValue;
  const dim3 grid = xcd_grid(a.Ho / SR, B, a.Cout / (16 * FC)), blk(MPI * 2);
  if (a.res_mode != 0 && !a.gamma) return hipErrorInvalidValue;   // residual modes are ResnetBlock convs
  if constexpr (SH > 0) {                                 // residual mode and GroupNorm from the shape
    constexpr ConvShape c = kStripShapes[SH];
    hipLaunchKernelGGL((conv_strip_kernel<T, FC, W, CIN, MPI, c.res, c.gn != 0, SH>), grid, blk, lds, s, a, SR);
  } else if (a.res_mode == 0 && !a.gamma) hipLaunchKernelGGL((conv_strip_kernel<T, FC, W, CIN, MPI, 0, false, 0>), grid, blk, lds, s, a, SR);
  else if (a.res_mode == 0) hipLaunchKernelGGL((conv_strip_kernel<T, FC, W, CIN, MPI, 0, true, 0>), grid, blk, lds, s, a, SR);
  else if (a.res_mode == 1) hipLaunchKernelGGL((conv_strip_kernel<T, FC, W, CIN, MPI, 1, true, 0>), grid, blk, lds, s, a, SR);
  else hipLaunchKernelGGL((conv_strip_kernel<T, FC, W, CIN, MPI, 2, true, 0>), grid, blk, lds, s, a, SR);
  return hipGetLastError();
}

// mpi: pixels per iteration (128 -> 4 waves, 256 -> 8 waves = two per SIMD)
// the specialised shapes SH = 1 .. kNStripShapes-1 (16-bit storage only) matching the launch
template <typename T, int SH>
static bool strip_shape_go(const ConvArgs& a, int nblk, int mpi, int SR, int B, hipStream_t s, hipError_t& e) {
  if constexpr (SH >= kNStripShapes || sizeof(T) == 4) {
    return false;
  } else if constexpr (!shape_for_type<T>(kStripShapes[SH])) {
    return strip_shape_go<T, SH + 1>(a, nblk, mpi, SR, B, s, e);
  } else {
    constexpr ConvShape c = kStripShapes[SH];
    if (strip_shape_matches(c, nblk, mpi, SR, a)) {
      e = strip_go<T, c.cfg / 16, c.Wo, c.CA + c.CB, c.nw, SH>(a, SR, B, s, nullptr);
      return true;
    }
    return strip_shape_go<T, SH + 1>(a, nblk, mpi, SR, B, s, e);
  }
}

template <typename T>
hipError_t strip_dispatch(const ConvArgs& a, int nblk, int mpi, int SR, int B, hipStream_t s, size_t* lo) {
  static const bool generic = std::getenv("SDDM_NO_STRIP_SHAPES") != nullptr;   // A/B runs
  hipError_t e;
  if (!lo && !generic && strip_shape_go<T, 1>(a, nblk, mpi, SR, B, s, e)) return e;
  const int Cin = a.CA + a.CB;
#define SDDM_STRIP(FCV, WV, CV)                                                                   \
  if (nblk == 16 * FCV && a.Wo == WV && Cin == CV)                                                \
    return mpi == 256 ? strip_go<T, FCV, WV, CV, 256>(a, SR, B, s, lo) : strip_go<T, FCV, WV, CV, 128>(a, SR, B, s, lo);
  SDDM_STRIP(2, 128, 32) SDDM_STRIP(2, 128, 64) SDDM_STRIP(4, 128, 32) SDDM_STRIP(4, 128, 64)
  SDDM_STRIP(2, 64, 32) SDDM_STRIP(2, 64, 64) SDDM_STRIP(2, 64, 128)
  SDDM_STRIP(4, 64, 32) SDDM_STRIP(4, 64, 64) SDDM_STRIP(4, 64, 128)
#undef SDDM_STRIP
  if (lo) *lo = (size_t)1 << 40;
  return hipErrorInvalidValue;
}

}  // namespace sddm
