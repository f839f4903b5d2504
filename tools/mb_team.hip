// Probe of the team kernel's hand-off protocol (conv_deep.hip conv_team_kernel) with trivial work:
// 512 workgroups of 256 threads; a workgroup reads HW_REG_XCC_ID, joins that XCD's ticket queue
// (op-major tickets over L ops x 2 images x I items), waits for the previous op of its image
// (relaxed agent-scope sc1 poll, bounded by iterations AND s_memrealtime), reads the previous op's
// payload with sc1 buffer loads, writes its own slice with plain stores, drains, barrier, one
// agent-scope atomic add.  Reports: workgroups per XCC id, timeouts, stale words, time per op.
//   hipcc -O3 --offload-arch=gfx950 tools/mb_team.hip -o tools/_mb_team && ./tools/_mb_team
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct P {
  unsigned* ctr;      // [8][32] tickets, then done[L][16]
  unsigned* stat;     // [0] timeouts, [1] stale, [2..9] wgs per xcc, [10] max poll iterations
  unsigned* buf;      // payload [L + 1][16 images][I items][64 words]
  const char* arena;  // base of buf (sc1 buffer loads)
  int L, I, spin_mode;
};

__global__ __launch_bounds__(256, 2) void k_team(P p) {
  __shared__ int s_t;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  xcc &= 7;
  if (threadIdx.x == 0) atomicAdd(p.stat + 2 + xcc, 1u);
  const int B = 16, nimg = 2;
  unsigned* ticket = p.ctr + xcc * 32;
  unsigned* done = p.ctr + 256;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)p.arena, (short)0, -1, 0x00020000);
  for (;;) {
    // wave-uniform branches only around the barriers (a lane-0 branch here is structurised into a
    // lane-divergent loop around the barriers): wave 0 takes the ticket, its lane 0 adding 1
    const bool w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
    if (w0) s_t = (int)__builtin_amdgcn_readfirstlane(
        __hip_atomic_fetch_add(ticket, (threadIdx.x & 63) == 0 ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    __syncthreads();
    int t = __builtin_amdgcn_readfirstlane(s_t);
    const int per_op = nimg * p.I;
    const int op = t / per_op;
    if (op >= p.L) break;
    t -= op * per_op;
    const int j = t / p.I, item = t - j * p.I;
    const int b = (int)xcc + 8 * j;
    if (op > 0) {
      // the whole first wave polls with a wave-uniform (scalar) loop: a divergent lane-0 loop inside
      // the ticket loop is structurised into an exec-mask loop around the barriers and hangs
      if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0) {
        unsigned* c = done + (op - 1) * B + b;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned it = 0;
        for (;;) {
          const unsigned v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
          if (v >= (unsigned)p.I) break;
          if (p.spin_mode) __builtin_amdgcn_s_sleep(1);
          ++it;
          if (it > 2000000u || __builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {
            atomicAdd(p.stat, (threadIdx.x & 63) == 0 ? 1u : 0u);
            break;
          }
        }
        atomicMax(p.stat + 10, it);
      }
      asm volatile("s_barrier" ::: "memory");
    }
    // read every item of the previous op for this image (64 words each), check the tags
    unsigned stale = 0;
    if (op > 0)
      for (int w = threadIdx.x; w < p.I * 64; w += 256) {
        const unsigned off = (unsigned)((((op - 1) * 16 + b) * p.I * 64 + w) * 4 + (size_t)0);
        const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 16);
        if (v != (unsigned)(op << 16 | b << 8 | (w >> 6))) ++stale;
      }
    if (stale) atomicAdd(p.stat + 1, stale);
    if (threadIdx.x < 64) p.buf[((op * 16 + b) * p.I + item) * 64 + threadIdx.x] = (unsigned)((op + 1) << 16 | b << 8 | item);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (w0) __hip_atomic_fetch_add(done + op * B + b, (threadIdx.x & 63) == 0 ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int main() {
  P p{};
  p.L = 20; p.I = 32;
  const size_t nbuf = (size_t)(p.L + 1) * 16 * p.I * 64;
  CK(hipMalloc(&p.ctr, sizeof(unsigned) * (256 + p.L * 16)));
  CK(hipMalloc(&p.stat, sizeof(unsigned) * 16));
  CK(hipMalloc(&p.buf, sizeof(unsigned) * nbuf));
  p.arena = (const char*)p.buf;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int mode : {1, 0}) {
    p.spin_mode = mode;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipMemset(p.ctr, 0, sizeof(unsigned) * (256 + p.L * 16)));
      CK(hipMemset(p.stat, 0, sizeof(unsigned) * 16));
      CK(hipMemset(p.buf, 0xff, sizeof(unsigned) * nbuf));
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k_team, dim3(512), dim3(256), 0, 0, p);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipDeviceSynchronize());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned st[16];
      CK(hipMemcpy(st, p.stat, sizeof(st), hipMemcpyDeviceToHost));
      printf("sleep=%d rep %d: %.2f us/op  timeouts %u stale %u max poll iters %u  wgs per xcc:", mode, rep,
             ms * 1e3f / p.L, st[0], st[1], st[10]);
      for (int x = 0; x < 8; ++x) printf(" %u", st[2 + x]);
      printf("\n");
      fflush(stdout);
    }
  }
  printf("MB_TEAM_OK\n");
  return 0;
}
