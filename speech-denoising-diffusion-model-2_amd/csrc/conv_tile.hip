// Tile implicit-GEMM 3x3 convolution with K split across waves, for the narrow UNet levels
// (segment width <= 32: 64x32 ... 8x4 images with 64..320 channels) and the stride-2 Downsample
// convolutions (UNetModified2.py:103-109).  Deep levels have few output pixels, so an M-only
// decomposition leaves most of the 256 CUs idle; here the 4 waves of a block are arranged as
// WM x KW (WM * KW = 4): waves with the same wm share pixels, waves with the same wk take every
// KW-th 32-channel K chunk.  Each round the block stages KW transformed input chunks (GroupNorm +
// SiLU, nearest upsample and channel concat applied while loading) in LDS, one per wk; the
// weight fragments come straight from L2 (they are read once per block).  ResnetBlock.res_conv
// 1x1 chunks (raw input, centre tap) join the same K distribution.  The KW partial tiles are
// reduced through LDS, then bias + embedding + identity residual are added, 4-channel vectors
// stored, and per-tile GroupNorm statistics written for the consumer.
#include "conv_common.h"
#include "kernels.h"

namespace sddm {

template <typename T, bool S2, int KW, int FP, int FC, int MAXU>
__global__ __launch_bounds__(256) void conv_tile_kernel(ConvArgs a) {
  constexpr int WM = 4 / KW;
  constexpr int ES = (int)sizeof(T);
  constexpr int CK = 32;
  constexpr int PIX = CK * ES + 16;   // LDS bytes per staged pixel chunk
  constexpr int MBLK = WM * FP * 16, NBLK = FC * 16;
  constexpr int UPP = CK * ES / 16;
  constexpr int VE = 16 / ES;
  constexpr int LG = 8 * ES;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int wm = wave / KW, wk = wave - wm * KW;
  const int tile = blockIdx.x, b = blockIdx.y, n0 = blockIdx.z * NBLK;
  const int ty = tile / a.tiles_x, tx = tile - ty * a.tiles_x;
  const int y0 = ty * a.TR, x0 = tx * a.TW;
  const int HR = S2 ? 2 * a.TR + 1 : a.TR + 2, HC = S2 ? 2 * a.TW + 1 : a.TW + 2;
  const int Cin = a.CA + a.CB, nck = Cin / CK;
  const int RC = a.RCA + a.RCB, rck = a.res_mode == 2 ? RC / CK : 0;
  const int nall = nck + rck;
  const bool gn = a.gamma != nullptr;
  const int npix_valid = a.TR * a.TW;
  const int slot_bytes = ((HR * HC > MBLK ? HR * HC : MBLK) * PIX + 15) & ~15;

  char* stage = smem;                                   // [KW][slot]
  float* gsc = (float*)(stage + KW * slot_bytes);       // [2][Cin]
  if (gn) {
    const GNFuse f{a.gstA, a.gtilesA, a.gntileA, a.gstB, a.gtilesB, a.gntileB, a.gamma, a.beta, a.groups, a.eps};
    gn_fused_prologue(f, b, a.CA, a.CB, gsc, gsc + Cin);
  }

  int pix_off[FP], pix_lin[FP];
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    int p = wm * FP * 16 + fp * 16 + (lane & 15);
    if (p >= npix_valid) p = 0;
    const int py = p / a.TW, px = p - py * a.TW;
    pix_off[fp] = ((S2 ? 2 * py : py) * HC + (S2 ? 2 * px : px)) * PIX + g * LG;
    pix_lin[fp] = p * PIX + g * LG;
  }
  f32x4 acc[FP][FC];
#pragma unroll
  for (int i = 0; i < FP; ++i)
#pragma unroll
    for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const size_t img_in = (size_t)a.Hi * a.Wi;
  const int rounds = (nall + KW - 1) / KW;
  const int halo_units = HR * HC * UPP;             // units of one 3x3 chunk
  for (int rd = 0; rd < rounds; ++rd) {
    // ---- 1. this wave's weight fragments for the whole chunk (latency overlaps the staging) ----
    const int myck = rd * KW + wk;
    constexpr bool PRE = KW > 1;       // K-split blocks are few: hide the weight latency behind staging
    constexpr int NW = PRE ? 9 : 1;
    Frag<T> wf[NW][FC];
    if (PRE && myck < nck) {
      const T* wrow = (const T*)a.wgt + ((size_t)(n0 + (lane & 15)) * nck + myck) * 9 * CK + g * 8;
      const size_t fstride = (size_t)16 * nck * 9 * CK;   // 16 output channels
#pragma unroll
      for (int tap = 0; tap < NW; ++tap)
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) wf[tap][fc] = load_frag<T>((const char*)(wrow + fc * fstride + tap * CK));
    } else if (myck >= nck && myck < nall) {
      const int c0 = (myck - nck) * CK;
#pragma unroll
      for (int fc = 0; fc < FC; ++fc)
        wf[0][fc] = load_frag<T>((const char*)((const T*)a.res_wgt + (size_t)(n0 + fc * 16 + (lane & 15)) * RC + c0 + g * 8));
    }
    if constexpr (PRE) {
    // ---- 2. batched staging loads of chunks rd*KW .. rd*KW+KW-1 (all 256 threads) ----
    const int nst = min(KW, nall - rd * KW);
    int total = 0;
    for (int s = 0; s < nst; ++s) total += (rd * KW + s < nck) ? halo_units : MBLK * UPP;
    f32x4 reg[MAXU];
    int dst[MAXU];                                    // LDS byte offset, -1 = nothing
    int gsel[MAXU];                                   // channel offset for the GN affine, -1 = no transform
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * 256;
      dst[k] = -1;
      gsel[k] = -1;
      reg[k] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (u >= total) continue;
      int s = 0, v = u;
      while (s < nst) {
        const int n = (rd * KW + s < nck) ? halo_units : MBLK * UPP;
        if (v < n) break;
        v -= n;
        ++s;
      }
      const int ck = rd * KW + s;
      char* slot = stage + s * slot_bytes;
      if (ck < nck) {
        const int c0 = ck * CK;
        const int hp = v / UPP, q = v - hp * UPP;
        const int hy = hp / HC, hx = hp - hy * HC;
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
        dst[k] = (int)(slot - smem) + hp * PIX + q * 16;
        if (ok) {
          const bool fromA = c0 < a.CA;
          const T* src = fromA ? (const T*)a.srcA : (const T*)a.srcB;
          const int Cs = fromA ? a.CA : a.CB;
          const size_t pi = (size_t)b * img_in + (size_t)iy * a.Wi + ix;
          reg[k] = *(const f32x4*)((const char*)(src + pi * Cs + (fromA ? c0 : c0 - a.CA)) + q * 16);
          gsel[k] = c0 + q * VE;
        }
      } else {
        const int c0 = (ck - nck) * CK;
        const int p = v / UPP, q = v - p * UPP;
        dst[k] = (int)(slot - smem) + p * PIX + q * 16;
        if (p < npix_valid) {
          const bool fromA = c0 < a.RCA;
          const T* src = fromA ? (const T*)a.rawA : (const T*)a.rawB;
          const int Cs = fromA ? a.RCA : a.RCB;
          const int py = p / a.TW, px = p - py * a.TW;
          const size_t pi = ((size_t)b * a.Ho + (y0 + py)) * a.Wo + (x0 + px);
          reg[k] = *(const f32x4*)((const char*)(src + pi * Cs + (fromA ? c0 : c0 - a.RCA)) + q * 16);
        }
      }
    }
    __syncthreads();   // previous round's readers done (and gsc written on the first round)
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      if (dst[k] < 0) continue;
      f32x4 v = reg[k];
      if (gn && gsel[k] >= 0) v = transform_fast<T>(v, gsc + gsel[k], gsc + Cin + gsel[k]);
      *(f32x4*)(smem + dst[k]) = v;
    }
    for (int u = tid + MAXU * 256; u < total; u += 256) {   // overflow (never for the planned shapes)
      int s = 0, v = u;
      while (s < nst) {
        const int n = (rd * KW + s < nck) ? halo_units : MBLK * UPP;
        if (v < n) break;
        v -= n;
        ++s;
      }
      const int ck = rd * KW + s;
      char* slot = stage + s * slot_bytes;
      if (ck < nck) {
        const int c0 = ck * CK, hp = v / UPP, q = v - hp * UPP, hy = hp / HC, hx = hp - hy * HC;
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
        f32x4 val = {0.f, 0.f, 0.f, 0.f};
        if (ok) {
          const bool fromA = c0 < a.CA;
          const T* src = fromA ? (const T*)a.srcA : (const T*)a.srcB;
          const int Cs = fromA ? a.CA : a.CB;
          const size_t pi = (size_t)b * img_in + (size_t)iy * a.Wi + ix;
          val = *(const f32x4*)((const char*)(src + pi * Cs + (fromA ? c0 : c0 - a.CA)) + q * 16);
          if (gn) val = transform_fast<T>(val, gsc + c0 + q * VE, gsc + Cin + c0 + q * VE);
        }
        *(f32x4*)(slot + hp * PIX + q * 16) = val;
      } else {
        const int c0 = (ck - nck) * CK, p = v / UPP, q = v - p * UPP;
        f32x4 val = {0.f, 0.f, 0.f, 0.f};
        if (p < npix_valid) {
          const bool fromA = c0 < a.RCA;
          const T* src = fromA ? (const T*)a.rawA : (const T*)a.rawB;
          const int Cs = fromA ? a.RCA : a.RCB;
          const int py = p / a.TW, px = p - py * a.TW;
          const size_t pi = ((size_t)b * a.Ho + (y0 + py)) * a.Wo + (x0 + px);
          val = *(const f32x4*)((const char*)(src + pi * Cs + (fromA ? c0 : c0 - a.RCA)) + q * 16);
        }
        *(f32x4*)(slot + p * PIX + q * 16) = val;
      }
    }
    __syncthreads();
    } else {
    // ---- 2'. streaming staging (KW == 1: many resident blocks hide the latency, keep VGPRs low) ----
    __syncthreads();
    {
      const int ck = rd;
      char* slot = stage;
      if (ck < nck) {
        const int c0 = ck * CK;
        const bool fromA = c0 < a.CA;
        const T* src = fromA ? (const T*)a.srcA : (const T*)a.srcB;
        const int Cs = fromA ? a.CA : a.CB;
        const int cs0 = fromA ? c0 : c0 - a.CA;
        const int rowu = HC * UPP;
        int hy = tid / rowu, j = tid - hy * rowu;
        for (int u = tid; u < halo_units; u += 256) {
          const int hx = j / UPP, q = j - hx * UPP, hp = hy * HC + hx;
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
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (ok) {
            const size_t pi = (size_t)b * img_in + (size_t)iy * a.Wi + ix;
            v = *(const f32x4*)((const char*)(src + pi * Cs + cs0) + q * 16);
            if (gn) v = transform_fast<T>(v, gsc + c0 + q * VE, gsc + Cin + c0 + q * VE);
          }
          *(f32x4*)(slot + hp * PIX + q * 16) = v;
          j += 256;
          while (j >= rowu) { j -= rowu; ++hy; }
        }
      } else {
        const int c0 = (ck - nck) * CK;
        const bool fromA = c0 < a.RCA;
        const T* src = fromA ? (const T*)a.rawA : (const T*)a.rawB;
        const int Cs = fromA ? a.RCA : a.RCB;
        const int cs0 = fromA ? c0 : c0 - a.RCA;
        for (int u = tid; u < MBLK * UPP; u += 256) {
          const int p = u / UPP, q = u - p * UPP;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (p < npix_valid) {
            const int py = p / a.TW, px = p - py * a.TW;
            const size_t pi = ((size_t)b * a.Ho + (y0 + py)) * a.Wo + (x0 + px);
            v = *(const f32x4*)((const char*)(src + pi * Cs + cs0) + q * 16);
          }
          *(f32x4*)(slot + p * PIX + q * 16) = v;
        }
      }
    }
    __syncthreads();
    }
    // ---- 3. this wave's chunk ----
    if (myck < nall) {
      const char* slot = stage + wk * slot_bytes;
      if (myck < nck) {
        const T* wrow = (const T*)a.wgt + ((size_t)(n0 + (lane & 15)) * nck + myck) * 9 * CK + g * 8;
        const size_t fstride = (size_t)16 * nck * 9 * CK;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int dy = tap / 3, dx = tap - 3 * dy;
          const int toff = (dy * HC + dx) * PIX;
          Frag<T> af[FC];
#pragma unroll
          for (int fc = 0; fc < FC; ++fc)
            af[fc] = PRE ? wf[PRE ? tap : 0][fc] : load_frag<T>((const char*)(wrow + fc * fstride + tap * CK));
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) {
            const Frag<T> bf = load_frag<T>(slot + pix_off[fp] + toff);
#pragma unroll
            for (int fc = 0; fc < FC; ++fc) mfma_frag(acc[fp][fc], af[fc], bf);
          }
        }
      } else {
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) {
          const Frag<T> bf = load_frag<T>(slot + pix_lin[fp]);
#pragma unroll
          for (int fc = 0; fc < FC; ++fc) mfma_frag(acc[fp][fc], wf[0][fc], bf);
        }
      }
    }
  }
  __syncthreads();
  // ---- reduce the KW partial tiles through LDS: red[wk][MBLK][NBLK+1] ----
  constexpr int OLD = NBLK + 1;
  float* red = (float*)smem;
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    const int p = wm * FP * 16 + fp * 16 + (lane & 15);
#pragma unroll
    for (int fc = 0; fc < FC; ++fc)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[(wk * MBLK + p) * OLD + fc * 16 + 4 * g + i] = acc[fp][fc][i];
  }
  __syncthreads();
  const int t_now = a.t_dev ? *a.t_dev : 0;
  const float* trow = a.temb ? a.temb + (size_t)(a.temb_per_b ? b : t_now) * a.temb_ld : nullptr;
  const int nco = min(NBLK, a.Cout - n0);
  float* ot = red + (size_t)KW * MBLK * OLD;   // final tile [MBLK][OLD]
  for (int u = tid; u < npix_valid * (NBLK / 4); u += 256) {
    const int p = u / (NBLK / 4), c4 = (u - p * (NBLK / 4)) * 4;
    if (c4 >= nco) continue;
    const int py = p / a.TW, px = p - py * a.TW;
    const size_t po = ((size_t)b * a.Ho + (y0 + py)) * a.Wo + (x0 + px);
    float v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < KW; ++k) s += red[(k * MBLK + p) * OLD + c4 + i];
      const int co = n0 + c4 + i;
      v[i] = s + a.bias[co] + (trow ? trow[co] : 0.f);
    }
    if (a.res_mode == 1) {
      const f32x4 r = load4<T>((const T*)a.res_src + po * a.Cout + n0 + c4);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += r[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = round_t<T>(v[i]);
      ot[p * OLD + c4 + i] = v[i];
    }
    store4<T>((T*)a.out + po * a.Cout + n0 + c4, v[0], v[1], v[2], v[3]);
  }
  if (a.stats) {
    __syncthreads();
    tile_channel_stats(ot, OLD, npix_valid, nco, a.stats + (((size_t)b * a.n_tiles + tile) * a.Cout + n0) * 2, 2);
  }
}

template <typename T, bool S2, int KW, int FP, int FC>
static size_t tile_lds(const ConvArgs& a) {
  constexpr int ES = (int)sizeof(T), PIX = 32 * ES + 16;
  constexpr int WM = 4 / KW, MBLK = WM * FP * 16, NBLK = FC * 16;
  const int HR = S2 ? 2 * a.TR + 1 : a.TR + 2, HC = S2 ? 2 * a.TW + 1 : a.TW + 2;
  const size_t slot = ((size_t)(HR * HC > MBLK ? HR * HC : MBLK) * PIX + 15) & ~(size_t)15;
  const size_t stage = KW * slot + (size_t)2 * (a.CA + a.CB) * 4;
  const size_t epi = (size_t)(KW + 1) * MBLK * (NBLK + 1) * 4;
  return stage > epi ? stage : epi;
}

template <typename T, bool S2, int KW, int FP, int FC>
static hipError_t tile_launch(const ConvArgs& a, int B, hipStream_t s, size_t* lo) {
  const size_t lds = tile_lds<T, S2, KW, FP, FC>(a);
  if (lo) { *lo = lds; return hipSuccess; }
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int nz = (a.Cout + FC * 16 - 1) / (FC * 16);
  // staging units per round -> register array size
  constexpr int UPP = 32 * (int)sizeof(T) / 16;
  const int HR = S2 ? 2 * a.TR + 1 : a.TR + 2, HC = S2 ? 2 * a.TW + 1 : a.TW + 2;
  const int units = KW * HR * HC * UPP;
  const int per = (units + 255) / 256;
  const dim3 grid(a.n_tiles, B, nz);
  if (per <= 4) hipLaunchKernelGGL((conv_tile_kernel<T, S2, KW, FP, FC, 4>), grid, dim3(256), lds, s, a);
  else if (per <= 8) hipLaunchKernelGGL((conv_tile_kernel<T, S2, KW, FP, FC, 8>), grid, dim3(256), lds, s, a);
  else hipLaunchKernelGGL((conv_tile_kernel<T, S2, KW, FP, FC, 16>), grid, dim3(256), lds, s, a);
  return hipGetLastError();
}

template <typename T>
static hipError_t tile_dispatch(const ConvCfg& c, const ConvArgs& a, int B, hipStream_t s, size_t* lo) {
#define SDDM_TILE(S2V, KWV, FPV)                                       \
  if (c.stride2 == S2V && c.kw == KWV && c.fp == FPV && c.nblk == 32) \
    return tile_launch<T, S2V, KWV, FPV, 2>(a, B, s, lo);
  SDDM_TILE(0, 4, 2) SDDM_TILE(0, 4, 4) SDDM_TILE(0, 4, 8) SDDM_TILE(0, 2, 2) SDDM_TILE(0, 2, 4)
  SDDM_TILE(0, 1, 1) SDDM_TILE(0, 1, 2)
  SDDM_TILE(1, 4, 2) SDDM_TILE(1, 4, 4) SDDM_TILE(1, 4, 8) SDDM_TILE(1, 2, 2) SDDM_TILE(1, 2, 4)
  SDDM_TILE(1, 1, 1) SDDM_TILE(1, 1, 2)
#undef SDDM_TILE
  return hipErrorInvalidValue;
}

hipError_t launch_conv3x3(int dtype, const ConvCfg& cfg, const ConvArgs& a, int B, hipStream_t s) {
  if (dtype == DT_F32) return tile_dispatch<float>(cfg, a, B, s, nullptr);
  if (dtype == DT_BF16) return tile_dispatch<bf16_t>(cfg, a, B, s, nullptr);
  return tile_dispatch<f16_t>(cfg, a, B, s, nullptr);
}

size_t conv3x3_lds_bytes(int dtype, const ConvCfg& cfg, const ConvArgs& a) {
  size_t lo = (size_t)1 << 40;
  if (dtype == DT_F32) (void)tile_dispatch<float>(cfg, a, 1, 0, &lo);
  else if (dtype == DT_BF16) (void)tile_dispatch<bf16_t>(cfg, a, 1, 0, &lo);
  else (void)tile_dispatch<f16_t>(cfg, a, 1, 0, &lo);
  return lo;
}

}  // namespace sddm
