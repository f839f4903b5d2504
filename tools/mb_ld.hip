// Load latency probe: per workgroup, a 64 KB region written with plain stores and drained, then
// (a) 16 16-byte loads per lane in flight, sc1 buffer loads vs plain global loads, and (b) a
// 64-long dependent chain of 4-byte loads by one lane, sc1 vs plain.  s_memrealtime (100 MHz).
//   hipcc -O3 --offload-arch=gfx950 tools/mb_ld.hip -o tools/_mb_ld && ./tools/_mb_ld
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k(char* base, unsigned long long* out, int nwg_active) {
  if ((int)blockIdx.x >= nwg_active) return;
  const int tid = threadIdx.x;
  char* reg = base + (size_t)blockIdx.x * 3 * 65536;
  unsigned* chain = (unsigned*)(reg + 2 * 65536);
  // write 2 x 64 KB of payload and a pointer chain (4 KB stride)
  for (int i = tid; i < 2 * 4096; i += 256) ((f32x4*)reg)[i] = f32x4{1.f, 2.f, 3.f, (float)i};
  if (tid < 16) chain[tid * 1024] = (unsigned)(((tid + 1) & 15) * 1024);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)reg, (short)0, -1, 0x00020000);
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  f32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 16; ++j)
    acc += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (unsigned)((j * 256 + tid) * 16), 0, 16));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  const f32x4* p2 = (const f32x4*)(reg + 65536);
#pragma unroll
  for (int j = 0; j < 16; ++j) acc += p2[j * 256 + tid];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
  unsigned idx = 0, idx2 = 0;
  if (__builtin_amdgcn_readfirstlane(tid >> 6) == 0) {
    for (int j = 0; j < 64; ++j)
      idx = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_raw_buffer_load_b32(rs, 2 * 65536 + idx * 4, 0, 16));
  }
  __syncthreads();
  unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
  if (__builtin_amdgcn_readfirstlane(tid >> 6) == 0) {
    for (int j = 0; j < 64; ++j) idx2 = __builtin_amdgcn_readfirstlane(((volatile unsigned*)chain)[idx2]);
  }
  __syncthreads();
  unsigned long long t4 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {
    out[blockIdx.x * 4 + 0] = t1 - t0;
    out[blockIdx.x * 4 + 1] = t2 - t1;
    out[blockIdx.x * 4 + 2] = t3 - t2;
    out[blockIdx.x * 4 + 3] = t4 - t3 + (idx + idx2 + (unsigned)acc.x == 12345u);
  }
}

int main() {
  char* base;
  unsigned long long* out;
  CK(hipMalloc(&base, (size_t)512 * 3 * 65536));
  CK(hipMalloc(&out, 512 * 4 * 8));
  for (int n : {1, 64, 512}) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemset(out, 0, 512 * 32));
      hipLaunchKernelGGL(k, dim3(512), dim3(256), 0, 0, base, out, n);
      CK(hipDeviceSynchronize());
    }
    unsigned long long h[512 * 4];
    CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
    double s[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < 4; ++j) s[j] += h[i * 4 + j];
    printf("%3d workgroups: 64 KB sc1 %.2f us, 64 KB plain %.2f us, 64 dependent sc1 loads %.2f us (%.0f ns each), 64 dependent volatile %.2f us\n",
           n, s[0] / n / 100, s[1] / n / 100, s[2] / n / 100, s[2] / n / 100 / 64 * 1000, s[3] / n / 100);
    fflush(stdout);
  }
  printf("MB_LD_OK\n");
  return 0;
}
