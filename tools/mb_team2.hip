// Staged probe of the team-kernel protocol pieces (each stage printed before the next starts):
// A XCC_ID census, B s_memrealtime-bounded spin, C ticket queue only, D one dependency hop.
//   hipcc -O3 --offload-arch=gfx950 tools/mb_team2.hip -o tools/_mb_team2 && ./tools/_mb_team2
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x;
}

__global__ void kA(unsigned* hist) {
  if (threadIdx.x == 0) atomicAdd(hist + (xcc_id() & 15), 1u);
}

__global__ void kB(unsigned long long* out) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned n = 0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < 100000ull) { __builtin_amdgcn_s_sleep(1); ++n; }   // 1 ms
    out[0] = __builtin_amdgcn_s_memrealtime() - t0;
    out[1] = n;
  }
}

__global__ __launch_bounds__(256, 2) void kC(unsigned* ctr, unsigned* per, int total) {
  __shared__ int s_t;
  const unsigned x = xcc_id() & 7;
  int mine = 0;
  for (;;) {
    if (threadIdx.x == 0) s_t = (int)__hip_atomic_fetch_add(ctr + x * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int t = __builtin_amdgcn_readfirstlane(s_t);
    __syncthreads();
    if (t >= total) break;
    ++mine;
  }
  if (threadIdx.x == 0) atomicAdd(per + x, (unsigned)mine);
}

// D: the first half of each team's workgroups add to a counter, the second half wait for it
__global__ __launch_bounds__(256, 2) void kD(unsigned* ctr, unsigned* res) {
  const unsigned x = xcc_id() & 7;
  __shared__ int s_t;
  if (threadIdx.x == 0) s_t = (int)__hip_atomic_fetch_add(ctr + x * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int t = __builtin_amdgcn_readfirstlane(s_t);
  unsigned* done = ctr + 256 + x * 32;
  if (t < 32) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned n = 0;
    bool to = false;
    while (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 32u) {
      __builtin_amdgcn_s_sleep(1);
      if (++n > 100000u || __builtin_amdgcn_s_memrealtime() - t0 > 1000000ull) { to = true; break; }
    }
    atomicAdd(res + (to ? 1 : 0), 1u);
    atomicMax(res + 2, n);
  }
}

int main() {
  unsigned *hist, *ctr, *per, *res;
  unsigned long long* tb;
  CK(hipMalloc(&hist, 64)); CK(hipMalloc(&ctr, 4096 * 4)); CK(hipMalloc(&per, 64)); CK(hipMalloc(&res, 64)); CK(hipMalloc(&tb, 16));
  CK(hipMemset(hist, 0, 64));
  hipLaunchKernelGGL(kA, dim3(512), dim3(256), 0, 0, hist);
  CK(hipDeviceSynchronize());
  unsigned h[16];
  CK(hipMemcpy(h, hist, 64, hipMemcpyDeviceToHost));
  printf("A xcc census:"); for (int i = 0; i < 16; ++i) printf(" %u", h[i]); printf("\n"); fflush(stdout);
  hipLaunchKernelGGL(kB, dim3(1), dim3(64), 0, 0, tb);
  CK(hipDeviceSynchronize());
  unsigned long long b[2];
  CK(hipMemcpy(b, tb, 16, hipMemcpyDeviceToHost));
  printf("B 1 ms spin: %llu ticks, %llu sleeps\n", b[0], b[1]); fflush(stdout);
  CK(hipMemset(ctr, 0, 4096 * 4)); CK(hipMemset(per, 0, 64));
  hipLaunchKernelGGL(kC, dim3(512), dim3(256), 0, 0, ctr, per, 1280);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h, per, 32, hipMemcpyDeviceToHost));
  printf("C tickets per team:"); for (int i = 0; i < 8; ++i) printf(" %u", h[i]); printf("\n"); fflush(stdout);
  CK(hipMemset(ctr, 0, 4096 * 4)); CK(hipMemset(res, 0, 64));
  hipLaunchKernelGGL(kD, dim3(512), dim3(256), 0, 0, ctr, res);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h, res, 12, hipMemcpyDeviceToHost));
  printf("D waits ok %u timed out %u max polls %u\n", h[0], h[1], h[2]); fflush(stdout);
  printf("MB_TEAM2_OK\n");
  return 0;
}
