// Row-streaming ("line buffer") 3x3 convolution for the wide UNet levels (segment width W = 128
// and 64: UNetModified2 levels 0-1, where >60 % of the FLOPs live).
//
// One block owns image b, output channels [n0, n0 + 16*FC) and a strip of SR output rows.  It
// keeps in LDS
//   * the whole weight slab of its channel tile (loaded once per strip, not once per tile), and
//   * a ring of R = 2*TR + 2 transformed input rows (GroupNorm + SiLU applied once per element,
//     zero halo columns, nearest-2x upsample / channel concat resolved while loading),
// and walks the strip TR = 128 / W output rows at a time (128 pixels = 4 waves x 2 MFMA column
// fragments).  While the MFMAs of iteration i run on rows [y-1, y+TR] of the ring, each thread
// already holds in registers the raw input of rows [y+TR+1, y+2TR] (issued before the MFMAs) and
// writes them transformed into the free ring slots afterwards: one barrier per iteration.
// The epilogue adds bias, the noise-embedding projection and the residual (identity, or the
// ResnetBlock 1x1 res_conv as extra MFMAs on raw input fragments loaded straight to registers),
// stores 4 channels per lane, and accumulates GroupNorm statistics of the stored values in
// registers (per-lane shifted sums, merged with Chan's formula at the end of the strip).
#include "conv_common.h"
#include "kernels.h"

namespace sddm {

template <typename T, int FC, int MAXU>
__global__ __launch_bounds__(256) void conv_strip_kernel(ConvArgs a, int TR, int SR) {
  constexpr int FP = 2;
  constexpr int ES = (int)sizeof(T);
  constexpr int NBLK = 16 * FC;
  constexpr int LG = 8 * ES;        // bytes of a lane group's 8 channels
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int strip = blockIdx.x, b = blockIdx.y, n0 = blockIdx.z * NBLK;
  const int W = a.Wo, H = a.Ho;
  const int Cin = a.CA + a.CB, nck = Cin / 32;
  const int R = 2 * TR + 2;
  const int PIXB = Cin * ES + 16;
  const int SLOT = (W + 2) * PIXB;
  const int WROW = nck * 9 * 32 * ES + 16;
  const int RC = a.RCA + a.RCB;
  const int RROW = RC * ES + 16;
  const bool gn = a.gamma != nullptr;
  const bool res2 = a.res_mode == 2;
  const int UPP = Cin * ES / 16;    // 16-byte units per pixel
  const int VE = 16 / ES;

  char* ring = smem;
  char* wl = ring + R * SLOT;
  char* rw = wl + NBLK * WROW;
  float* gsc = (float*)(rw + (res2 ? NBLK * RROW : 0));
  float* red = gsc + 2 * Cin;       // [4 waves][NBLK][3]

  const int y0 = strip * SR;
  // ---------------- prologue ----------------
  if (gn) {
    const GNFuse f{a.gstA, a.gtilesA, a.gntileA, a.gstB, a.gtilesB, a.gntileB, a.gamma, a.beta, a.groups, a.eps};
    gn_fused_prologue(f, b, a.CA, a.CB, gsc, gsc + Cin);
  }
  {
    const int upr = (WROW - 16) / 16;
    for (int u = tid; u < NBLK * upr; u += 256) {
      const int row = u / upr, q = u - row * upr;
      *(f32x4*)(wl + row * WROW + q * 16) =
          *(const f32x4*)((const char*)a.wgt + (size_t)(n0 + row) * (WROW - 16) + q * 16);
    }
    if (res2) {
      const int rpr = RC * ES / 16;
      for (int u = tid; u < NBLK * rpr; u += 256) {
        const int row = u / rpr, q = u - row * rpr;
        *(f32x4*)(rw + row * RROW + q * 16) =
            *(const f32x4*)((const char*)a.res_wgt + ((size_t)(n0 + row) * RC) * ES + q * 16);
      }
    }
    // zero halo columns of every slot
    for (int u = tid; u < R * 2 * UPP; u += 256) {
      const int s = u / (2 * UPP), rem = u - s * 2 * UPP, side = rem / UPP, q = rem - side * UPP;
      *(f32x4*)(ring + s * SLOT + (side ? (W + 1) : 0) * PIXB + q * 16) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __syncthreads();

  // raw 16-byte unit of output-space input row ry, column x, channel unit q (zero outside the image)
  auto load_unit = [&](int ry, int x, int q) -> f32x4 {
    if (ry < 0 || ry >= H) return f32x4{0.f, 0.f, 0.f, 0.f};
    int sy = ry, sx = x;
    if (a.upsample) { sy >>= 1; sx >>= 1; }
    const size_t pix = ((size_t)b * a.Hi + sy) * a.Wi + sx;
    const int c0 = q * VE;
    if (c0 < a.CA) return *(const f32x4*)((const T*)a.srcA + pix * a.CA + c0);
    return *(const f32x4*)((const T*)a.srcB + pix * a.CB + (c0 - a.CA));
  };
  auto row_valid = [&](int ry) { return ry >= 0 && ry < H; };

  // initial rows y0-1 .. y0+TR
  {
    const int n = (TR + 2) * W * UPP;
    for (int u = tid; u < n; u += 256) {
      const int p = u / UPP, q = u - p * UPP, r = p / W, x = p - r * W;
      const int ry = y0 - 1 + r;
      const f32x4 raw = load_unit(ry, x, q);
      const f32x4 v = row_valid(ry) ? transform_vec<T>(raw, gsc + q * VE, gsc + Cin + q * VE, gn) : raw;
      const int slot = ((ry % R) + R) % R;
      *(f32x4*)(ring + slot * SLOT + (x + 1) * PIXB + q * 16) = v;
    }
  }
  __syncthreads();

  // per-lane pixel geometry inside an iteration (128 pixels = TR rows x W)
  int prow[FP], pcol[FP];
#pragma unroll
  for (int fp = 0; fp < FP; ++fp) {
    const int p = wave * 32 + fp * 16 + (lane & 15);
    prow[fp] = p / W;
    pcol[fp] = p - prow[fp] * W;
  }
  // running GroupNorm statistics (shift K = first value seen)
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

  const int iters = SR / TR;
  const int npre = TR * W * UPP;    // units of the TR rows prefetched per iteration
  for (int it = 0; it < iters; ++it) {
    const int y = y0 + it * TR;
    // ---- issue the prefetch of rows y+TR+1 .. y+2TR (raw) ----
    f32x4 pre[MAXU];
    const bool do_pre = it + 1 < iters;
#pragma unroll
    for (int k = 0; k < MAXU; ++k) {
      const int u = tid + k * 256;
      if (do_pre && u < npre) {
        const int p = u / UPP, q = u - p * UPP, r = p / W, x = p - r * W;
        pre[k] = load_unit(y + TR + 1 + r, x, q);
      }
    }
    // ---- MFMA over the 9 taps x Cin/32 chunks of the current rows ----
    f32x4 acc[FP][FC];
#pragma unroll
    for (int i = 0; i < FP; ++i)
#pragma unroll
      for (int j = 0; j < FC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int rowoff[FP][3];
#pragma unroll
    for (int fp = 0; fp < FP; ++fp)
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) {
        const int ry = y + prow[fp] + dy - 1;
        rowoff[fp][dy] = (((ry % R) + R) % R) * SLOT + pcol[fp] * PIXB + g * LG;
      }
    const char* wbase = wl + (lane & 15) * WROW + g * LG;
    for (int ck = 0; ck < nck; ++ck) {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3, dx = tap - 3 * dy;
        Frag<T> bf[FP];
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) bf[fp] = load_frag<T>(ring + rowoff[fp][dy] + dx * PIXB + ck * 32 * ES);
#pragma unroll
        for (int fc = 0; fc < FC; ++fc) {
          const Frag<T> af = load_frag<T>(wbase + fc * 16 * WROW + (ck * 9 + tap) * 32 * ES);
#pragma unroll
          for (int fp = 0; fp < FP; ++fp) mfma_frag(acc[fp][fc], af, bf[fp]);
        }
      }
    }
    if (res2) {  // ResnetBlock.res_conv 1x1 on the raw block input, B fragments straight from global
      const char* rbase = rw + (lane & 15) * RROW + g * LG;
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
          const Frag<T> af = load_frag<T>(rbase + fc * 16 * RROW + ck * 32 * ES);
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
      for (int k = 0; k < MAXU; ++k) {
        const int u = tid + k * 256;
        if (u < npre) {
          const int p = u / UPP, q = u - p * UPP, r = p / W, x = p - r * W;
          const int ry = y + TR + 1 + r;
          const f32x4 v = row_valid(ry) ? transform_vec<T>(pre[k], gsc + q * VE, gsc + Cin + q * VE, gn) : pre[k];
          *(f32x4*)(ring + (((ry % R) + R) % R) * SLOT + (x + 1) * PIXB + q * 16) = v;
        }
      }
    }
    __syncthreads();
  }

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
      for (int w = 0; w < 4; ++w) {
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
}

template <typename T, int FC>
static size_t strip_lds(const ConvArgs& a, int TR) {
  constexpr int ES = (int)sizeof(T), NBLK = 16 * FC;
  const int Cin = a.CA + a.CB;
  const int R = 2 * TR + 2;
  size_t n = (size_t)R * (a.Wo + 2) * (Cin * ES + 16) + (size_t)NBLK * ((Cin / 32) * 9 * 32 * ES + 16);
  if (a.res_mode == 2) n += (size_t)NBLK * ((a.RCA + a.RCB) * ES + 16);
  n += (size_t)2 * Cin * 4 + (size_t)4 * NBLK * 3 * 4;
  return n;
}

template <typename T>
static hipError_t strip_dispatch(const ConvArgs& a, int nblk, int SR, int B, hipStream_t s, size_t* lds_only) {
  const int TR = 128 / a.Wo;
  const size_t lds = nblk == 64 ? strip_lds<T, 4>(a, TR) : strip_lds<T, 2>(a, TR);
  if (lds_only) { *lds_only = lds; return hipSuccess; }
  const int Cin = a.CA + a.CB;
  const int units = TR * a.Wo * Cin * (int)sizeof(T) / 16;
  if (lds > 160 * 1024 || a.Wo * TR != 128 || a.Ho % SR || SR % TR || units > 16 * 256 || Cin % 32)
    return hipErrorInvalidValue;
  const int nz = (a.Cout + nblk - 1) / nblk;
  dim3 grid(a.Ho / SR, B, nz);
  const int upt = (units + 255) / 256;
#define SDDM_STRIP(FCV, UV)                                                                        \
  hipLaunchKernelGGL((conv_strip_kernel<T, FCV, UV>), grid, dim3(256), lds, s, a, TR, SR);
  if (nblk == 64) {
    if (upt <= 2) { SDDM_STRIP(4, 2) } else if (upt <= 4) { SDDM_STRIP(4, 4) } else if (upt <= 8) { SDDM_STRIP(4, 8) } else { SDDM_STRIP(4, 16) }
  } else {
    if (upt <= 2) { SDDM_STRIP(2, 2) } else if (upt <= 4) { SDDM_STRIP(2, 4) } else if (upt <= 8) { SDDM_STRIP(2, 8) } else { SDDM_STRIP(2, 16) }
  }
#undef SDDM_STRIP
  return hipGetLastError();
}

hipError_t launch_conv_strip(int dtype, int nblk, int SR, const ConvArgs& a, int B, hipStream_t s) {
  if (dtype == DT_F32) return strip_dispatch<float>(a, nblk, SR, B, s, nullptr);
  if (dtype == DT_BF16) return strip_dispatch<bf16_t>(a, nblk, SR, B, s, nullptr);
  return strip_dispatch<f16_t>(a, nblk, SR, B, s, nullptr);
}

size_t conv_strip_lds_bytes(int dtype, int nblk, const ConvArgs& a) {
  size_t lo = 0;
  if (dtype == DT_F32) (void)strip_dispatch<float>(a, nblk, 1, 1, 0, &lo);
  else if (dtype == DT_BF16) (void)strip_dispatch<bf16_t>(a, nblk, 1, 1, 0, &lo);
  else (void)strip_dispatch<f16_t>(a, nblk, 1, 1, 0, &lo);
  return lo;
}

}  // namespace sddm
