// LDS-DMA (global_load_lds_dwordx4) issue and landing time by lane address pattern (round-5 probe:
// the deep kernel's halo DMAs give each lane a different pixel, 64 cache lines per instruction).
// 256 workgroups x 8 waves, each wave issues NL DMAs of 1 KiB into its own LDS slab, then
// s_waitcnt vmcnt(0).  Patterns: coalesced (lane l -> base + 16 l), stride320 (lane l -> base +
// 320 l, a 160-channel bf16 pixel row per lane), block8 (8 lanes = 8 consecutive 16-B units of one
// pixel row, 8 pixel rows per instruction), quad4 (4 lanes = 4 consecutive units of one pixel
// row, 16 rows per instruction: the round-6 deep halo), unitmaj (16 lanes = one unit of 16 rows).
// L2-warm: every workgroup reads the same 512 KiB.
//   hipcc -O3 --offload-arch=gfx950 tools/mb_dma.hip -o tools/_mb_dma && ./tools/_mb_dma
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int NL, int PAT>
__global__ __launch_bounds__(512) void k_dma(const char* __restrict__ src, unsigned long long* st) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char* base = src + wave * 8192;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const char* p;
    if (PAT == 0) p = base + k * 1024 + lane * 16;
    else if (PAT == 1) p = base + (k % 20) * 16 + lane * 320 + (k / 20) * 64 * 320;
    else if (PAT == 2) p = base + (lane >> 3) * 320 + ((k % 2) * 8 + (lane & 7)) * 16 + (k / 2) * 8 * 320;
    else if (PAT == 3) p = base + (lane >> 2) * 320 + ((k % 5) * 4 + (lane & 3)) * 16 + (k / 5) * 16 * 320;
    else p = base + (lane & 15) * 320 + ((k % 5) * 4 + (lane >> 4)) * 16 + (k / 5) * 16 * 320;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)p,
                                     (__attribute__((address_space(3))) void*)(smem + wave * (NL * 1024) + k * 1024), 16, 0, 0);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { st[blockIdx.x * 4] = t0; st[blockIdx.x * 4 + 1] = t1; st[blockIdx.x * 4 + 2] = t2; }
}

template <int NL, int PAT>
static int run(const char* name, const char* src, unsigned long long* st, hipStream_t s) {
  const int G = 256;
  double mi = 0, mt = 0;
  int n = 0;
  for (int rep = 0; rep < 6; ++rep) {
    hipLaunchKernelGGL((k_dma<NL, PAT>), dim3(G), dim3(512), 8 * NL * 1024, s, src, st);
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(G * 4);
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    if (rep < 2) continue;
    for (int b = 0; b < G; ++b) { mi += (h[b * 4 + 1] - h[b * 4]) * 1e-2; mt += (h[b * 4 + 2] - h[b * 4]) * 1e-2; ++n; }
  }
  printf("%-10s NL %2d (%3d KiB per CU): issue %.2f us, landed %.2f us\n", name, NL, NL * 8, mi / n, mt / n);
  return 0;
}

int main() {
  char* src;
  unsigned long long* st;
  CK(hipMalloc(&src, 64 << 20)); CK(hipMemset(src, 0, 64 << 20));
  CK(hipMalloc(&st, 256 * 4 * 8));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
#define RUN(NL, PAT, NAME) if (run<NL, PAT>(NAME, src, st, s)) return 1;
  RUN(4, 0, "coalesced") RUN(8, 0, "coalesced") RUN(16, 0, "coalesced")
  RUN(4, 1, "stride320") RUN(8, 1, "stride320") RUN(16, 1, "stride320")
  RUN(4, 2, "block8") RUN(8, 2, "block8") RUN(16, 2, "block8")
  RUN(4, 3, "quad4") RUN(8, 3, "quad4") RUN(16, 3, "quad4")
  RUN(4, 4, "unitmaj") RUN(8, 4, "unitmaj") RUN(16, 4, "unitmaj")
  printf("MB_OK\n");
  return 0;
}
