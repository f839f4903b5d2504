// Row-streaming ("line buffer") 3x3 convolution for the wide UNet levels (segment width W = 128
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
// stores 4 channels per lane, and accumulates GroupNorm statistics of the stored values in
// registers (per-lane shifted sums, merged with Chan's formula at the end of the strip).
#include "conv_common.h"
#include "kernels.h"

namespace sddm {

template <typename T, int FC, int W, int CIN, int MPI>
__global__ __launch_bounds__(MPI * 2) void conv_strip_kernel(ConvArgs a, int SR) {
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
  constexpr int UPT = NU / NT;                    // prefetch units per thread
  static_assert(UPP >= 1 && UPP <= 64 && (64 % UPP) == 0, "channel units must divide a wave");
  static_assert(NU % NT == 0, "prefetch must split evenly");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int strip = blockIdx.x, b = blockIdx.y, n0 = blockIdx.z * NBLK;
  const int H = a.Ho;
  const int RC = a.RCA + a.RCB;
  const bool gn = a.gamma != nullptr;
  const bool res2 = a.res_mode == 2;

  char* ring = smem;                              // [R][UPP planes][PL]
  char* wl = ring + R * SLOT;                     // [WPLANES][NBLK][16 B]
  char* rw = wl + WPLANES * WPL;                  // [RC*ES/16 planes][NBLK][16 B]
  const int RPLANES = res2 ? RC * ES / 16 : 0;
  float* gsc = (float*)(rw + RPLANES * WPL);      // [2][CIN]
  float* red = gsc + 2 * CIN;                     // [NWV waves][NBLK][3]

  const int y0 = strip * SR;
  SDDM_STAMP(a, 0);
  // ---------------- prologue ----------------
  if (gn) {
    const GNFuse f{a.gstA, a.gtilesA, a.gntileA, a.gstB, a.gtilesB, a.gntileB, a.gamma, a.beta, a.groups, a.eps};
    gn_fused_prologue(f, b, a.CA, a.CB, gsc, gsc + CIN);
  }
  for (int u = tid; u < NBLK * WPLANES; u += NT) {        // co fastest: conflict-free LDS writes
    const int co = u % NBLK, pl = u / NBLK;                 // pl = (ck*9 + tap)*4*UPL + unit
    const int ck = pl / (9 * 4 * UPL), rem = pl - ck * 9 * 4 * UPL, tap = rem / (4 * UPL), un = rem - tap * 4 * UPL;
    *(f32x4*)(wl + pl * WPL + co * 16) =
        *(const f32x4*)((const char*)a.wgt + ((((size_t)(n0 + co) * NCK + ck) * 9 + tap) * 32) * ES + un * 16);
  }
  if (res2) {
    for (int u = tid; u < NBLK * RPLANES; u += NT) {
      const int co = u % NBLK, pl = u / NBLK;
      *(f32x4*)(rw + pl * WPL + co * 16) = *(const f32x4*)((const char*)a.res_wgt + ((size_t)(n0 + co) * RC) * ES + pl * 16);
    }
  }
  for (int u = tid; u < R * UPP * 2; u += NT) {           // zero halo columns
    const int side = u & 1, pl = u >> 1;
    *(f32x4*)(ring + pl * PL + (side ? (W + 1) : 0) * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();                                         // gsc ready

  auto load_unit = [&](int ry, int x, int q) -> f32x4 {
    if (ry < 0 || ry >= H) return f32x4{0.f, 0.f, 0.f, 0.f};
    int sy = ry, sx = x;
    if (a.upsample) { sy >>= 1; sx >>= 1; }
    const size_t pix = ((size_t)b * a.Hi + sy) * a.Wi + sx;
    const int c0 = q * VE;
    if (c0 < a.CA) return *(const f32x4*)((const T*)a.srcA + pix * a.CA + c0);
    return *(const f32x4*)((const T*)a.srcB + pix * a.CB + (c0 - a.CA));
  };
  const int base = ((y0 - 1) % R + R) % R;                 // ring slot of row y0 - 1

  // initial rows y0-1 .. y0+TR
  for (int u = tid; u < (TR + 2) * W * UPP; u += NT) {
    const int grp = u >> 6, j = u & 63;
    const int pix = grp * PB + (j % PB), q = j / PB, r = pix / W, x = pix % W;
    const int ry = y0 - 1 + r;
    f32x4 v = load_unit(ry, x, q);
    if (gn && ry >= 0 && ry < H) v = transform_fast<T>(v, gsc + q * VE, gsc + CIN + q * VE);
    *(f32x4*)(ring + ((base + r) % R) * SLOT + q * PL + (x + 1) * 16) = v;
  }
  __syncthreads();
  SDDM_STAMP(a, 3);

  int prow[FP], pcol[FP];
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    const int p = wave * 32 + fp * 16 + (lane & 15);   // pixel inside the MPI-pixel iteration
    prow[fp] = p / W;
    pcol[fp] = p % W;
  }
  // prefetch geometry of this thread's units (same every iteration): source pointer of row 0
  // (column and channel offset folded in) and the unit's row inside the TR-row group
  int pr[UPT], px[UPT], pq[UPT];
  const char* ubase[UPT];
  int ustride[UPT];
#pragma unroll
  for (int k = 0; k < UPT; ++k) {
    const int u = tid + k * NT, grp = u >> 6, j = u & 63;
    const int pix = grp * PB + (j % PB);
    pq[k] = j / PB;
    pr[k] = pix / W;
    px[k] = pix % W;
    const int c0 = pq[k] * VE;
    const int sx = a.upsample ? (px[k] >> 1) : px[k];
    const bool fa = c0 < a.CA;
    const int Cs = fa ? a.CA : a.CB;
    ubase[k] = (const char*)((fa ? (const T*)a.srcA : (const T*)a.srcB) +
                             (((size_t)b * a.Hi) * a.Wi + sx) * Cs + (fa ? c0 : c0 - a.CA));
    ustride[k] = a.Wi * Cs * ES;                           // bytes per source row
  }
  float sK[FC][4], s1[FC][4], s2[FC][4];
#pragma unroll
  for (int fc = 0; fc < FC; ++fc)
#pragma unroll
    for (int i = 0; i < 4; ++i) { sK[fc][i] = 0.f; s1[fc][i] = 0.f; s2[fc][i] = 0.f; }
  const int t_now = a.t_dev ? *a.t_dev : 0;
  const float* trow = a.temb ? a.temb + (size_t)(a.temb_per_b ? b : t_now) * a.temb_ld : nullptr;
  float badd[FC][4];
#pragma unroll
  for (int fc = 0; fc < FC; ++fc)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = n0 + fc * 16 + 4 * g + i;
      badd[fc][i] = (co < a.Cout) ? a.bias[co] + (trow ? trow[co] : 0.f) : 0.f;
    }
  const char* abase = wl + g * UPL * WPL + (lane & 15) * 16;
  const char* rbase = rw + g * UPL * WPL + (lane & 15) * 16;

  const int iters = SR / TR;
  for (int it = 0; it < iters; ++it) {
    const int y = y0 + it * TR;
    const int s_it = (base + it * TR) % R;                 // slot of row y - 1
    // ---- issue the prefetch of rows y+TR+1 .. y+2TR (raw) ----
    f32x4 pre[UPT];
    const bool do_pre = it + 1 < iters;
    if (do_pre) {
#pragma unroll
      for (int k = 0; k < UPT; ++k) {
        const int ry = y + TR + 1 + pr[k];
        const int sy = a.upsample ? (ry >> 1) : ry;
        pre[k] = ry < H ? *(const f32x4*)(ubase[k] + sy * ustride[k]) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    // ---- MFMA over the 9 taps x CIN/32 chunks of the current rows ----
    f32x4 acc[FP][FC];
#pragma unroll
    for (int i = 0; i < FP; ++i)
#pragma unroll
      for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* bptr[FP][3];
#pragma unroll
    for (int fp = 0; fp < FP; ++fp)
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
        bptr[fp][dy] = ring + ((s_it + prow[fp] + dy) % R) * SLOT + g * UPL * PL + pcol[fp] * 16;
#pragma unroll
    for (int ck = 0; ck < NCK; ++ck) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3, dx = tap - 3 * dy;
        Frag<T> bf[FP];
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) bf[fp] = load_planes<T>(bptr[fp][dy] + ck * 4 * UPL * PL + dx * 16, PL);
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) {
          const Frag<T> af = load_planes<T>(abase + (ck * 9 + tap) * 4 * UPL * WPL + fc * 256, WPL);
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) mfma_frag(acc[fp][fc], af, bf[fp]);
        }
      }
    }
    if (res2) {  // ResnetBlock.res_conv 1x1 on the raw block input, B fragments straight from global
      for (int ck = 0; ck < RC / 32; ++ck) {
        Frag<T> bf[FP];
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) {
          const size_t pix = ((size_t)b * H + y + prow[fp]) * W + pcol[fp];
          const int c0 = ck * 32 + g * 8;
          const T* sp = c0 < a.RCA ? (const T*)a.rawA + pix * a.RCA + c0 : (const T*)a.rawB + pix * a.RCB + (c0 - a.RCA);
          bf[fp] = load_frag<T>((const char*)sp);
        }
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) {
          const Frag<T> af = load_planes<T>(rbase + ck * 4 * UPL * WPL + fc * 256, WPL);
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) mfma_frag(acc[fp][fc], af, bf[fp]);
        }
      }
    }
    // ---- epilogue: bias + embedding + residual, store, statistics ----
#pragma unroll
    for (int fp = 0; fp < FP; ++fp) {
      const size_t po = ((size_t)b * H + y + prow[fp]) * W + pcol[fp];
#pragma unroll
      for (int fc = 0; fc < FC; ++fc) {
        const int co = n0 + fc * 16 + 4 * g;
        if (co >= a.Cout) continue;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[fp][fc][i] + badd[fc][i];
        if (a.res_mode == 1) {
          const f32x4 r = load4<T>((const T*)a.res_src + po * a.Cout + co);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] += r[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = round_t<T>(v[i]);
        store4<T>((T*)a.out + po * a.Cout + co, v[0], v[1], v[2], v[3]);
        if (it == 0 && fp == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i) sK[fc][i] = v[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float d = v[i] - sK[fc][i];
          s1[fc][i] += d;
          s2[fc][i] += d * d;
        }
      }
    }
    // ---- transform the prefetched rows into the free ring slots ----
    if (do_pre) {
#pragma unroll
      for (int k = 0; k < UPT; ++k) {
        const int ry = y + TR + 1 + pr[k];
        f32x4 v = pre[k];
        if (gn && ry < H) v = transform_fast<T>(v, gsc + pq[k] * VE, gsc + CIN + pq[k] * VE);
        *(f32x4*)(ring + ((s_it + TR + 2 + pr[k]) % R) * SLOT + pq[k] * PL + (px[k] + 1) * 16) = v;
      }
    }
    __syncthreads();
  }

  SDDM_STAMP(a, 4);
  // ---- GroupNorm statistics of the strip: lanes -> waves -> block ----
  if (a.stats) {
    const float nl = (float)(FP * iters);
#pragma unroll
    for (int fc = 0; fc < FC; ++fc)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float n = nl;
        float mean = sK[fc][i] + s1[fc][i] / nl;
        float m2 = fmaxf(s2[fc][i] - s1[fc][i] * s1[fc][i] / nl, 0.f);
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {   // lanes with the same lane >> 4 hold the same channels
          const float mo = __shfl_xor(mean, o), m2o = __shfl_xor(m2, o);
          const float d = mo - mean;
          m2 = m2 + m2o + d * d * (n * 0.5f);
          mean = mean + 0.5f * d;
          n *= 2.f;
        }
        if ((lane & 15) == 0) {
          float* rr = red + ((wave * NBLK) + fc * 16 + 4 * g + i) * 3;
          rr[0] = n; rr[1] = mean; rr[2] = m2;
        }
      }
    __syncthreads();
    if (tid < NBLK && n0 + tid < a.Cout) {
      float n = 0.f, mean = 0.f, m2 = 0.f;
      for (int w = 0; w < NWV; ++w) {
        const float* rr = red + (w * NBLK + tid) * 3;
        const float nb = rr[0], d = rr[1] - mean, nt = n + nb;
        mean += d * nb / nt;
        m2 += rr[2] + d * d * n * nb / nt;
        n = nt;
      }
      float* dst = a.stats + (((size_t)b * a.n_tiles + strip) * a.Cout + n0 + tid) * 2;
      dst[0] = mean * n;
      dst[1] = m2;
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

template <typename T, int FC, int W, int CIN, int MPI>
static hipError_t strip_go(const ConvArgs& a, int SR, int B, hipStream_t s, size_t* lo) {
  const size_t lds = strip_lds<T, FC, W, CIN, MPI>(a);
  if (lo) { *lo = lds; return hipSuccess; }
  constexpr int TR = MPI / W;
  if (lds > 160 * 1024 || a.Ho % SR || SR % TR) return hipErrorInvalidValue;
  const int nz = (a.Cout + 16 * FC - 1) / (16 * FC);
  hipLaunchKernelGGL((conv_strip_kernel<T, FC, W, CIN, MPI>), dim3(a.Ho / SR, B, nz), dim3(MPI * 2), lds, s, a, SR);
  return hipGetLastError();
}

// mpi: pixels per iteration (128 -> 4 waves, 256 -> 8 waves = two per SIMD)
template <typename T>
static hipError_t strip_dispatch(const ConvArgs& a, int nblk, int mpi, int SR, int B, hipStream_t s, size_t* lo) {
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

hipError_t launch_conv_strip(int dtype, int nblk, int mpi, int SR, const ConvArgs& a, int B, hipStream_t s) {
  if (dtype == DT_F32) return strip_dispatch<float>(a, nblk, mpi, SR, B, s, nullptr);
  if (dtype == DT_BF16) return strip_dispatch<bf16_t>(a, nblk, mpi, SR, B, s, nullptr);
  return strip_dispatch<f16_t>(a, nblk, mpi, SR, B, s, nullptr);
}

size_t conv_strip_lds_bytes(int dtype, int nblk, int mpi, const ConvArgs& a) {
  size_t lo = (size_t)1 << 40;
  if (dtype == DT_F32) (void)strip_dispatch<float>(a, nblk, mpi, 1, 1, 0, &lo);
  else if (dtype == DT_BF16) (void)strip_dispatch<bf16_t>(a, nblk, mpi, 1, 1, 0, &lo);
  else (void)strip_dispatch<f16_t>(a, nblk, mpi, 1, 1, 0, &lo);
  return lo;
}

}  // namespace sddm
