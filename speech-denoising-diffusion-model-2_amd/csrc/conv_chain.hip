// Fused deep-level chain: the UNet levels whose images are 128 and 32 pixels (16x8 and 8x4 at
// num_samples 16448: downs.8 Downsample, downs.9 ResnetBlock, downs.10 Downsample, mid.0, ups.0
// ResnetBlock, ups.1 Upsample, ups.2 / ups.3 ResnetBlocks -- UNetModified2.py:93-142 modules in
// the UNetModified2.py:252-265 loops) as ONE launch with one workgroup per image.
//
// Why: per-layer launches at these levels are chains of dependent memory round trips (the
// producer's GroupNorm tile statistics, the input halo, the weights, the epilogue stores) over
// grids that cover a fraction of the chip; 13 of them cost ~160 us per reverse step while their
// arithmetic is 9 GFLOP.  Here an image's activations and GroupNorm statistics stay in LDS from
// op to op, the statistics are exact per image (no tile combination), and the memory traffic is
// the weight stream (shared by the images of an XCD through its L2), the chain's input and output,
// and the long-lived skip tensors the host planner parks in global memory between their uses.
//
// A workgroup is 4 waves, one per SIMD, each with the SIMD's whole register file: a wave owns
// all pixels of the image and NFW 16-channel output fragments (MFW x NFW accumulators), so no
// weight fragment is loaded twice per CU, and its weight ring holds the next 9 K steps (a
// whole 32-channel chunk, 9 x NFW KiB in flight per wave), which the L2 / MALL latency of the
// shared weight stream needs.
//
// Per op:
//   1. GroupNorm finalize from the producers' per-channel (mean, M2) in LDS (equal-count Chan
//      combination per group), scale / shift into LDS;
//   2. K loop over the flattened K steps (tap x 32-channel chunk of the 3x3 conv, then the 1x1
//      res_conv chunks of block2).  The 3x3 chunks are staged in groups of `nslot` (as many as
//      the LDS plan leaves room for): the GN + SiLU-transformed, zero-padded halo image (nearest-2x
//      upsample and stride-2 index maps, virtual concat), plane-major so the 16 lanes of an MFMA
//      operand read 16 consecutive 16-byte units.  The res_conv's raw input is read straight from
//      the LDS images (the planner keeps res_conv sources in LDS).  Weight fragments stream from
//      the fragment-major image through the ring (step s + 9 loaded right after step s's MFMAs);
//      the pixel fragments of step s + 1 are read from LDS while step s's MFMAs run.  Staging
//      happens only at chunk boundaries, so inside a chunk the memory counter holds nothing but
//      the weight stream;
//   3. epilogue: bias + noise embedding (+ identity residual), stores (LDS plane-major image and /
//      or global NHWC), exact two-pass per-channel statistics of the fp32 values (a wave holds all
//      pixels of its channels: DPP row sums, no LDS round trip) for the next op's GroupNorm.
// Reload ops copy a parked tensor from global memory back into an LDS image.
#include "conv_common.h"
#include "kernels.h"

namespace sddm {

// px, mfw, nfw (kept in sync with the dispatch in conv_chain_kernel)
static constexpr ChainVariant kChainVariants[] = {
    {128, 8, 2},   // 0: 128-pixel outputs, 5..8 channel fragments
    {128, 8, 3},   // 1: 128-pixel outputs, 9..12 channel fragments
    {32, 2, 2},    // 2: 32-pixel outputs, 5..8 channel fragments
    {32, 2, 3},    // 3: 32-pixel outputs, 9..12 channel fragments
};
int conv_chain_nvariants() { return (int)(sizeof(kChainVariants) / sizeof(kChainVariants[0])); }
ChainVariant conv_chain_variant(int v) { return kChainVariants[v]; }

namespace {

constexpr int kChainThreads = 256, kChainWaves = 4;

// pointers held in the descriptors are generic: loads / stores through them are issued as global
// (vmcnt only) instead of flat (which also counts against lgkmcnt, so every LDS wait would wait
// for the weight stream too)
#define SDDM_GLOBAL __attribute__((address_space(1)))
// the descriptors are read through the constant address space: uniform loads become scalar
// (s_load) loads into SGPRs, and every branch on them is a scalar branch
typedef const __attribute__((address_space(4))) ChainOp COp;
typedef const __attribute__((address_space(4))) ChainTensor CTen;
__device__ __forceinline__ f32x4 gload16(const void* p) { return *(const SDDM_GLOBAL f32x4*)p; }
__device__ __forceinline__ float gloadf(const float* p) { return *(const SDDM_GLOBAL float*)p; }
__device__ __forceinline__ void gstoref(float* p, float v) { *(SDDM_GLOBAL float*)p = v; }
template <typename T> __device__ __forceinline__ Frag<T> gload_frag(const void* p) {
  Frag<T> f;
  f.v = __builtin_bit_cast(decltype(f.v), gload16(p));
  return f;
}
template <typename T> __device__ __forceinline__ f32x4 gload4(const T* p) {   // 4 channels (8 bytes)
  typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
  typedef T t4 __attribute__((ext_vector_type(4)));
  const t4 v = __builtin_bit_cast(t4, *(const SDDM_GLOBAL u32x2_t*)p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
template <typename T> __device__ __forceinline__ void gstore4(T* p, float a0, float a1, float a2, float a3) {
  typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
  typedef T t4 __attribute__((ext_vector_type(4)));
  *(SDDM_GLOBAL u32x2_t*)p = __builtin_bit_cast(u32x2_t, t4{(T)a0, (T)a1, (T)a2, (T)a3});
}

// reload: tensor (global NHWC [P][C]) -> LDS plane-major image [C/8][P][8]
template <typename T>
__device__ __forceinline__ void chain_reload(COp& op, CTen* tens, char* smem, int b) {
  CTen& t = tens[op.a];
  const int C = t.C, H = t.H, W = t.W, P = H * W, cu = C >> 3, units = cu * P, dst = op.a_lds;
  const float rW = 1.0f / (float)W;
  const T* src = (const T*)t.g + (size_t)b * P * C;
  const float rcu = 1.0f / (float)cu;
  for (int u0 = 0; u0 < units; u0 += 4 * kChainThreads) {
    f32x4 v[4];
    int d[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {   // channel units fastest: a pixel's contiguous bytes
      const int u = min(u0 + (int)threadIdx.x + m * kChainThreads, units - 1);
      const int p = fdivi(u, rcu), q = u - p * cu;
      const int y = fdivi(p, rW), x = p - y * W;   // NHWC pixel -> column-major LDS unit x * H + y
      v[m] = gload16(src + (size_t)p * C + q * 8);
      d[m] = u0 + (int)threadIdx.x + m * kChainThreads < units ? dst + (q * P + x * H + y) * 16 : -1;
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
      if (d[m] >= 0) *(f32x4*)(smem + d[m]) = v[m];
  }
  __syncthreads();
}

// weight fragment of K step s, 16-channel block nf (a function, not a lambda: a closure holding the
// two base pointers would stay in scratch memory)
// Per-op parameters staged in LDS one op ahead: [gamma Cin][beta Cin][bias + noise embedding Cout]
// fp32 in one of two buffers (3 x cmax floats each) right after the GN scale / shift.  The loads
// for op `nx` are issued at the start of the op before it and stored at its end, so no op waits
// for a global round trip for its GroupNorm affine or epilogue constants.
constexpr int kPrmPerThread = 4;   // 3 x cmax <= 4 x 256 (cmax <= 341)
__device__ __forceinline__ void chain_prm_load(const ChainArgs& a, COp* ops, int nx, int trow, float (&v)[kPrmPerThread]) {
#pragma unroll
  for (int k = 0; k < kPrmPerThread; ++k) v[k] = 0.f;
  if (nx >= a.nops) return;
  COp& o = ops[nx];
  CTen* tens = (CTen*)a.tens;
  const int Cin = tens[o.a].C + (o.b >= 0 ? tens[o.b].C : 0), Cout = o.Cout;
  const float* trw = a.temb + (size_t)trow * a.temb_ld + o.toff;
#pragma unroll
  for (int k = 0; k < kPrmPerThread; ++k) {
    const int e = (int)threadIdx.x + k * kChainThreads;
    if (o.gn && e < Cin) v[k] = gloadf(o.gamma + e);
    else if (o.gn && e < 2 * Cin) v[k] = gloadf(o.beta + (e - Cin));
    else if (e >= 2 * Cin && e < 2 * Cin + Cout) {
      const int c = e - 2 * Cin;
      v[k] = gloadf(o.bias + c) + (o.temb ? gloadf(trw + c) : 0.f);
    }
  }
}
__device__ __forceinline__ void chain_prm_store(const ChainArgs& a, char* smem, int par, const float (&v)[kPrmPerThread]) {
  float* dst = (float*)(smem + a.gsc) + 2 * a.cmax + par * 3 * a.cmax;
#pragma unroll
  for (int k = 0; k < kPrmPerThread; ++k) {
    const int e = (int)threadIdx.x + k * kChainThreads;
    if (e < 3 * a.cmax) dst[e] = v[k];
  }
}

template <typename T, int MFW, int NFW, int FX>
__device__ __forceinline__ void chain_op(const ChainArgs& a, COp& op, CTen* tens, char* smem, int b, int trow,
                                         unsigned long long* stamp, int par, int nx) {
  constexpr int NT = kChainThreads, NG = kChainWaves, MAXU = 8, D = 9;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, l16 = lane & 15;
  const int ng = __builtin_amdgcn_readfirstlane(tid >> 6);

  // every descriptor field copied into a local scalar first (the staging code selects among them
  // field by field: a reference selecting one of several descriptors would live in scratch)
  CTen& TA = tens[op.a];
  CTen& TB = tens[op.b >= 0 ? op.b : op.a];
  CTen& TO = tens[op.out];
  CTen& RA = tens[op.ra >= 0 ? op.ra : op.a];
  CTen& RB = tens[op.rb >= 0 ? op.rb : (op.ra >= 0 ? op.ra : op.a)];
  const int A_lds = op.a_lds, A_H = TA.H, A_W = TA.W, A_C = TA.C, A_P = TA.H * TA.W, A_st = TA.st;
  const int B_lds = op.b_lds, B_H = TB.H, B_W = TB.W, B_C = TB.C, B_P = TB.H * TB.W, B_st = TB.st;
  const int RA_lds = op.ra_lds, RA_C = RA.C, RB_lds = op.rb_lds, RB_C = RB.C;
  const T* A_g = (const T*)TA.g;
  const T* B_g = (const T*)TB.g;
  const T* RA_g = (const T*)RA.g;
  const int O_lds = op.o_lds, O_st = TO.st, O_gw = op.o_gw;
  T* O_g = (T*)TO.g;
  float* O_gst = TO.gst;
  const int s2 = op.s2, up = op.up, gn = op.gn, res_mode = op.res_mode, Cout = op.Cout;
  const int PLB = op.PLB, stg = op.stg, nslot = op.nslot, SLOT = op.slot;
  const int CA = A_C, CB = op.b >= 0 ? B_C : 0, Cin = CA + CB;
  const int RCA = res_mode == 2 ? RA_C : 0, RCB = (res_mode == 2 && op.rb >= 0) ? RB_C : 0;
  const int nck = Cin >> 5, rck = (RCA + RCB) >> 5;
  const int Ho = TO.H, Wo = TO.W, P = Ho * Wo;
  const int Hi = TA.H, Wi = TA.W;
  // staged halo: stride 1: HR x HC (row stride HC padded); stride 2: four polyphase planes
  // (halo row / column parity) of HR x HC each, so a stride-2 tap reads a stride-1 window
  const int HR = op.HR, HC = op.HC, HPH = HR * HC, HP = s2 ? 4 * HPH : HPH;
  const float rHC = 1.0f / (float)HC, rHo = 1.0f / (float)Ho, rP = 1.0f / (float)P, rHPH = 1.0f / (float)HPH;
  float* gsc = (float*)(smem + a.gsc);
  const int cmax = a.cmax;
  const int dbg = a.dbg;

  // bias + noise embedding of this lane's epilogue channels: issued first, used at the end
  // this op's parameters (staged in LDS by the previous op); the next op's are loaded now
  const float* prm = (const float*)(smem + a.gsc) + 2 * cmax + par * 3 * cmax;
  float pnext[kPrmPerThread];
  chain_prm_load(a, (COp*)a.ops, nx, trow, pnext);

  // ---- weight fragments: [Cout/16][K steps][64 lanes][8]; K step s = 9 * chunk + tap for the
  // 3x3 chunks, then one step per 1x1 res_conv chunk.  A ring of the next 9 steps per wave (slot =
  // tap in the 3x3 loop); a fragment address is a uniform base (scalar) plus the lane's 16 bytes ----
  const int ns3 = nck * 9;
  const int loff = lane * 16;
  const char* w3[NFW];
  const char* w1[NFW];
#pragma unroll
  for (int j = 0; j < NFW; ++j) {
    const int nf = ng + NG * j;
    w3[j] = (const char*)op.wf + (size_t)nf * ns3 * 1024;
    w1[j] = (const char*)op.rwf + (size_t)nf * rck * 1024;
  }
  const int wmask = (dbg & 1) ? 0 : -1;   // ablation: every load hits the chunk's first fragment
  Frag<T> A[D][NFW];
#pragma unroll
  for (int t = 0; t < D; ++t)
#pragma unroll
    for (int j = 0; j < NFW; ++j) A[t][j] = gload_frag<T>(w3[j] + (t & wmask) * 1024 + loff);

  // ---- 1. GroupNorm finalize: one thread per channel (two passes over <= 512 channels), each
  // combining its group's per-channel (mean, M2) from LDS; gamma / beta loaded with the weights ----
  if (gn) {
    const int G = a.groups, cpg = Cin / G;
    float gm[2], bt[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = min(tid + h * NT, Cin - 1);
      gm[h] = prm[c];
      bt[h] = prm[Cin + c];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = tid + h * NT;
      if (c < Cin) {
        const int c0 = (c / cpg) * cpg;
        const bool fa = c0 < CA;
        const float* st = (const float*)(smem + (fa ? A_st : B_st)) + (fa ? c0 : c0 - CA) * 2;
        const float n = (float)(fa ? A_P : B_P);
        float m = 0.f;
        for (int k = 0; k < cpg; ++k) m += st[2 * k];
        m /= (float)cpg;
        float m2 = 0.f;
        for (int k = 0; k < cpg; ++k) {
          const float d = st[2 * k] - m;
          m2 += st[2 * k + 1] + n * d * d;
        }
        const float rstd = 1.0f / sqrtf(m2 / (n * (float)cpg) + a.eps);
        const float sc = gm[h] * rstd;
        gsc[c] = sc;
        gsc[cmax + c] = bt[h] - m * sc;
      }
    }
    lds_sync();
  }

  // ---- staging of 3x3 chunks [k0, k1) into the slots of the staging buffer: a thread owns one
  // staged halo pixel at a time (its source pixel decoded once) and walks the group's chunks and
  // 16-byte channel planes (uniform: one scalar branch per chunk for an LDS or a global source) ----
  auto stage = [=](int k0, int k1) __attribute__((always_inline)) {
    // captured members copied to locals: a conditional on two members of the closure would select
    // between their addresses, and the closure would stay in scratch memory
    const int a_lds = A_lds, b_lds = B_lds, a_c = A_C, b_c = B_C, a_h = A_H, a_w = A_W, a_p = A_P;
    const T *a_g = A_g, *b_g = B_g;
    // units (chunk, plane, halo pixel) flattened over all threads, halo pixels fastest: every wave
    // takes a share even when the halo is smaller than the workgroup (the 8 x 4 levels)
    const int cq_n = (k1 - k0) * 4, total = cq_n * HP;
    const float rHP = 1.0f / (float)HP;
    constexpr int SU = 4;           // units in flight per thread (loads first, then transforms)
    for (int u0 = tid; u0 < total; u0 += SU * NT) {
      f32x4 x[SU];
      int dst[SU], ch[SU];
#pragma unroll
      for (int m = 0; m < SU; ++m) {
        const int u = min(u0 + m * NT, total - 1);
        const int cq = fdivi(u, rHP), hp = u - cq * HP, cc = cq >> 2, q = cq & 3;
        int hy, hx;
        if (s2) {                   // polyphase plane ph = (row parity, column parity)
          const int ph = fdivi(hp, rHPH), r2 = hp - ph * HPH, a2 = fdivi(r2, rHC);
          hy = 2 * a2 + (ph >> 1);
          hx = 2 * (r2 - a2 * HC) + (ph & 1);
        } else {
          hy = fdivi(hp, rHC);
          hx = hp - hy * HC;
        }
        int iy = hy - 1, ix = hx - 1;
        bool ok;
        if (s2) ok = iy >= 0 && iy < Hi && ix >= 0 && ix < Wi;
        else {
          ok = iy >= 0 && iy < Ho && ix >= 0 && ix < Wo;
          if (up) { iy >>= 1; ix >>= 1; }
        }
        // LDS images are column-major (unit x * H + y), global tensors NHWC (pixel y * W + x)
        const int lpx = ok ? ix * a_h + iy : 0, gpx = ok ? iy * a_w + ix : 0;
        const int c0 = (k0 + cc) * 32;
        const bool fa = c0 < CA;
        const int src_lds = fa ? a_lds : b_lds, src_c = fa ? a_c : b_c, cs = fa ? c0 : c0 - CA;
        const T* src_g = fa ? (const T*)a_g : (const T*)b_g;   // prvalues: no select of addresses
        if (src_lds >= 0) x[m] = *(const f32x4*)(smem + src_lds + (((cs >> 3) + q) * a_p + lpx) * 16);
        else x[m] = gload16(src_g + ((size_t)b * a_p + gpx) * src_c + cs + q * 8);
        dst[m] = u0 + m * NT < total ? stg + cc * SLOT + q * PLB + hp * 16 : -1;
        ch[m] = ok ? c0 + q * 8 : -1;   // GN channel, -1: zero padding
      }
#pragma unroll
      for (int m = 0; m < SU; ++m) {
        f32x4 v = x[m];
        if (gn) v = transform_lds<T>(v, gsc + max(ch[m], 0), gsc + cmax + max(ch[m], 0));
        if (ch[m] < 0) v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (dst[m] >= 0) *(f32x4*)(smem + dst[m]) = v;
      }
    }
  };

  // this wave's output pixels: fragment i covers the column-major pixels q = 16 i + l16 (x = q / Ho,
  // y = q % Ho: one column of a 16-row image, two columns of an 8-row one); the host pads the staged
  // row stride HC (odd for 16 rows, 2 mod 4 for 8) so the 16 lanes of every tap's read hit 16
  // different 16-byte bank groups.  Fragment i = fragment 0 shifted by FX columns.
  const int poff0 = ((l16 % Ho) * HC + l16 / Ho) * 16;
  const int boff = g * PLB + poff0, roff = (g * P + l16) * 16;   // per-lane parts (vector)
  const int ra_lds = RA_lds, rb_lds = RB_lds;
  auto tap = [=](int t) __attribute__((always_inline)) {   // staged-unit offset of tap t (t constant)
    const int dy = t / 3, dx = t % 3;
    return s2 ? ((dy & 1) * 2 + (dx & 1)) * HPH + (dy >> 1) * HC + (dx >> 1) : dy * HC + dx;
  };
  auto load_b3 = [=](int slot, int t, Frag<T> (&Bf)[MFW]) __attribute__((always_inline)) {
    const char* S = smem + boff + (stg + slot * SLOT + tap(t) * 16);   // uniform part in parentheses
#pragma unroll
    for (int i = 0; i < MFW; ++i) Bf[i] = load_frag<T>(S + i * FX * 16);
  };
  auto load_b1 = [=](int r, Frag<T> (&Bf)[MFW]) __attribute__((always_inline)) {   // res_conv chunk r
    const int c0 = r * 32;
    const bool fa = c0 < RCA;
    const char* S = smem + roff + ((fa ? ra_lds : rb_lds) + ((fa ? c0 : c0 - RCA) >> 3) * P * 16);
#pragma unroll
    for (int i = 0; i < MFW; ++i) Bf[i] = load_frag<T>(S + i * 256);
  };

  f32x4 acc[MFW][NFW];
#pragma unroll
  for (int i = 0; i < MFW; ++i)
#pragma unroll
    for (int j = 0; j < NFW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mfmas = [&](const Frag<T> (&Aj)[NFW], const Frag<T> (&Bf)[MFW]) __attribute__((always_inline)) {
    if (dbg & 4) return;
#pragma unroll
    for (int j = 0; j < NFW; ++j)
#pragma unroll
      for (int i = 0; i < MFW; ++i) mfma_frag(acc[i][j], Aj[j], Bf[i]);
  };

  // ---- 2. K loop.  Pixel fragments double-buffered: step s + 1's are read into Bb[(s + 1) & 1]
  // before step s's MFMAs (on Bb[s & 1]) are issued, so the LDS latency hides behind them ----
  Frag<T> Bb[2][MFW];
  int k0 = 0, k1 = 0;              // staged group [k0, k1)
  for (int kb = 0; kb < nck; ++kb) {   // 3x3 chunks: 9 taps, compile-time
    if (kb == k1) {                 // the next group of chunks
      k0 = k1;
      k1 = min(k0 + nslot, nck);
      if (kb > 0) lds_sync();       // every wave is done with the previous group
      if (!(dbg & 2)) stage(k0, k1);
      lds_sync();
      if (stamp && kb == 0 && threadIdx.x == 0) stamp[1] = __builtin_amdgcn_s_memrealtime();
      load_b3(kb - k0, 0, Bb[0]);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t < 8) load_b3(kb - k0, t + 1, Bb[(t + 1) & 1]);
      else if (kb + 1 < k1) load_b3(kb + 1 - k0, 0, Bb[1]);
      else if (kb + 1 == nck && rck > 0) load_b1(0, Bb[1]);
      mfmas(A[t], Bb[t & 1]);
      // refill: the same tap of the next chunk, or res_conv chunk t after the last 3x3 chunk
      // (scalar selects, no branch around the load)
#pragma unroll
      for (int j = 0; j < NFW; ++j) {
        const char* nxt = kb + 1 < nck ? w3[j] + ((kb + 1) * 9 + t) * 1024
                                       : (rck > 0 ? w1[j] + min(t, rck - 1) * 1024 : w3[j] + (ns3 - 1) * 1024);
        A[t][j] = gload_frag<T>((wmask ? nxt : w3[j]) + loff);
      }
    }
#pragma unroll
    for (int i = 0; i < MFW; ++i) Bb[0][i] = Bb[1][i];
  }
  for (int rb = 0; rb < rck; rb += D) {   // 1x1 res_conv chunks, raw operands straight from LDS
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int r = rb + d;
      if (r + 1 < rck) load_b1(r + 1, Bb[(d + 1) & 1]);
      if (r < rck) mfmas(A[d], Bb[d & 1]);
#pragma unroll
      for (int j = 0; j < NFW; ++j) A[d][j] = gload_frag<T>((wmask ? w1[j] + min(r + D, rck - 1) * 1024 : w3[j]) + loff);
    }
#pragma unroll
    for (int i = 0; i < MFW; ++i) Bb[0][i] = Bb[1][i];
  }

  if (stamp && threadIdx.x == 0) stamp[2] = __builtin_amdgcn_s_memrealtime();
  // ---- 3. epilogue (acc becomes the fp32 output values) ----
#pragma unroll
  for (int j = 0; j < NFW; ++j) {
    const f32x4 bv = *(const f32x4*)(prm + 2 * Cin + (ng + NG * j) * 16 + 4 * g);   // bias + embedding
#pragma unroll
    for (int i = 0; i < MFW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] += bv[r];
  }
  if (res_mode == 1) {              // identity residual (ResnetBlock with dim == dim_out)
#pragma unroll
    for (int i = 0; i < MFW; ++i) {
      const int q = i * 16 + l16, qx = fdivi(q, rHo), p = (q - qx * Ho) * Wo + qx;   // LDS unit, NHWC pixel
#pragma unroll
      for (int j = 0; j < NFW; ++j) {
        const int co = (ng + NG * j) * 16 + 4 * g;
        f32x4 x;
        if (RA_lds >= 0) x = load4<T>((const T*)(smem + RA_lds + ((co >> 3) * P + q) * 16) + (co & 7));
        else x = gload4<T>(RA_g + ((size_t)b * P + p) * RA_C + co);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] += x[r];
      }
    }
  }
  // the output may reuse the LDS of this op's inputs (the planner's half-step lifetimes): every
  // wave must be done reading them
  lds_sync();
#pragma unroll
  for (int i = 0; i < MFW; ++i) {
    const int q = i * 16 + l16, qx = fdivi(q, rHo), p = (q - qx * Ho) * Wo + qx;   // LDS unit, NHWC pixel
#pragma unroll
    for (int j = 0; j < NFW; ++j) {
      const int co = (ng + NG * j) * 16 + 4 * g;
      if (O_lds >= 0)
        store4<T>((T*)(smem + O_lds + ((co >> 3) * P + q) * 16) + (co & 7), acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      if (O_gw)
        gstore4<T>(O_g + ((size_t)b * P + p) * Cout + co, acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
  if (O_st >= 0 || O_gst) {
    // exact two-pass per-channel statistics over the image: a wave holds every pixel of its
    // channels (16 per fragment, DPP row sums; the MFW fragments in registers)
#pragma unroll
    for (int j = 0; j < NFW; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < MFW; ++i) s += acc[i][j][r];
        const float mu = row_sum16(s) * rP;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < MFW; ++i) {
          const float d = acc[i][j][r] - mu;
          q += d * d;
        }
        q = row_sum16(q);
        const int co = (ng + NG * j) * 16 + 4 * g + r;
        if (l16 == 0) {
          if (O_st >= 0) {
            float* st = (float*)(smem + O_st) + co * 2;
            st[0] = mu;
            st[1] = q;
          }
          if (O_gst) {
            float* gs = O_gst + ((size_t)b * Cout + co) * 2;
            gstoref(gs, mu * (float)P);
            gstoref(gs + 1, q);
          }
        }
      }
    }
  }
  chain_prm_store(a, smem, par ^ 1, pnext);
  if (stamp && threadIdx.x == 0) stamp[3] = __builtin_amdgcn_s_memrealtime();
  // the next op reads this op's LDS image / statistics / its parameters and its global stores
  // (workgroup-scope release / acquire)
  __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(kChainThreads, 1) void conv_chain_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  const int t_now = a.t_dev ? *a.t_dev : 0;
  const int ng = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int trow = a.temb_per_b ? b : t_now;
  int par = 0;                      // parameter buffer of the current conv op
  {
    int nx = 0;
    while (nx < a.nops && ((COp*)a.ops)[nx].kind == 1) ++nx;
    float v[kPrmPerThread];
    chain_prm_load(a, (COp*)a.ops, nx, trow, v);
    chain_prm_store(a, smem, 0, v);
    __syncthreads();
  }
  for (int i = 0; i < a.nops; ++i) {
    COp& op = ((COp*)a.ops)[i];
    int nx = i + 1;                 // the next conv op (its parameters are staged by this one)
    while (nx < a.nops && ((COp*)a.ops)[nx].kind == 1) ++nx;
    unsigned long long* stamp = a.stamps ? a.stamps + (size_t)b * 64 + 4 * min(i, 15) : nullptr;
    if (stamp && threadIdx.x == 0) stamp[0] = __builtin_amdgcn_s_memrealtime();
    if (op.kind == 1) {
      chain_reload<T>(op, (CTen*)a.tens, smem, b);
      continue;
    }
    // a wave computes NFW or NFW - 1 channel fragments (the host picks the variant so that every
    // wave has one of the two); the count is a template argument, so no load or MFMA sits under a
    // branch
#define SDDM_CHAIN_OP(MFW, NFW)                                                                     \
  if (ng + kChainWaves * ((NFW) - 1) < (op.Cout >> 4))                                              \
    chain_op<T, MFW, NFW, (MFW == 8 ? 1 : 2)>(a, op, (CTen*)a.tens, smem, b, trow, stamp, par, nx);  \
  else                                                                                            \
    chain_op<T, MFW, (NFW) - 1, (MFW == 8 ? 1 : 2)>(a, op, (CTen*)a.tens, smem, b, trow, stamp, par, nx);
    switch (op.var) {
      case 0: SDDM_CHAIN_OP(8, 2) break;
      case 1: SDDM_CHAIN_OP(8, 3) break;
      case 2: SDDM_CHAIN_OP(2, 2) break;
      default: SDDM_CHAIN_OP(2, 3) break;
    }
#undef SDDM_CHAIN_OP
    par ^= 1;
  }
  if (a.stamps && threadIdx.x == 0) a.stamps[(size_t)b * 64 + 63] = __builtin_amdgcn_s_memrealtime();
}

}  // namespace

hipError_t launch_conv_chain(int dtype, const ChainArgs& a, int B, hipStream_t s) {
  if (a.lds_bytes > 160 * 1024 || a.nops <= 0) return hipErrorInvalidValue;
  if (dtype == DT_BF16) hipLaunchKernelGGL(conv_chain_kernel<bf16_t>, dim3(B), dim3(kChainThreads), a.lds_bytes, s, a);
  else if (dtype == DT_F16) hipLaunchKernelGGL(conv_chain_kernel<f16_t>, dim3(B), dim3(kChainThreads), a.lds_bytes, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace sddm
