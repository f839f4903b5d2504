// How long does a workgroup take to ISSUE and to RECEIVE a burst of 16-byte-per-lane loads, by
// lane address pattern (round-5 probe: the deep conv kernels spend 3-7 us between block start
// and "all loads issued").  256 workgroups x 8 waves, each lane issues NL global_load_dwordx4
// (checked in the ISA: all loads, the stamp, then one s_waitcnt vmcnt(0)).  Patterns:
//   coalesced   lane l reads base + 16 l (+ 1 KiB per load)
//   stride320   lane l reads base + 320 l (one 16-byte piece per pixel of a 160-channel bf16 row)
//   same        every lane reads the same 16 bytes
// Stamps s_memrealtime at entry, after the issue, after the wait.  cold: every workgroup reads
// its own 512 KiB of a 256 MiB buffer after a 512 MiB write (HBM); L2-warm: every workgroup
// reads the same 512 KiB, replayed (the XCD's L2), so only the CU-side path is measured.
//   hipcc -O3 --offload-arch=gfx950 tools/mb_issue.hip -o tools/_mb_issue && ./tools/_mb_issue
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int NL, int PAT>
__global__ __launch_bounds__(512) void k_burst(const char* __restrict__ src, unsigned long long* st, float* out, int shared) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // each workgroup owns a 512 KiB region
  const char* base = src + (shared ? 0 : (size_t)blockIdx.x * (512 << 10)) + wave * (PAT == 1 ? 64 * 320 : 1024);
  f4 r[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const char* p;
    if (PAT == 0) p = base + lane * 16 + k * 8192;
    else if (PAT == 1) p = base + lane * 320 + (k & 19) * 16 + (k / 20) * (8 * 64 * 320);
    else p = base;
    r[k] = *(const f4*)p;
  }
  asm volatile("" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
  for (int k = 0; k < NL; ++k) asm volatile("" :: "v"(r[k]));   // every loaded register is live
  if (threadIdx.x == 0) {
    st[blockIdx.x * 4 + 0] = t0; st[blockIdx.x * 4 + 1] = t1; st[blockIdx.x * 4 + 2] = t2;
  }
}

__global__ void k_dirty(float* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (float)i;
}

template <int NL, int PAT>
static int run(const char* name, const char* src, float* big, size_t nbig, unsigned long long* st, float* out, hipStream_t s,
               int warm) {
  const int G = 256;
  std::vector<double> iss, tot;
  for (int rep = 0; rep < 6; ++rep) {
    if (!warm) hipLaunchKernelGGL(k_dirty, dim3(1024), dim3(256), 0, s, big, nbig);   // evict
    hipLaunchKernelGGL((k_burst<NL, PAT>), dim3(G), dim3(512), 0, s, src, st, out, warm);
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(G * 4);
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    if (rep == 0) continue;
    for (int b = 0; b < G; ++b) {
      iss.push_back((h[b * 4 + 1] - h[b * 4]) * 1e-2);
      tot.push_back((h[b * 4 + 2] - h[b * 4]) * 1e-2);
    }
  }
  double mi = 0, mt = 0;
  for (size_t i = 0; i < iss.size(); ++i) { mi += iss[i]; mt += tot[i]; }
  mi /= iss.size(); mt /= tot.size();
  const double kb = NL * 512 * 16 / 1024.0;
  printf("%s %-10s NL %2d (%4.0f KiB per CU): issue %.2f us, all landed %.2f us (%.0f GB/s per CU)\n", warm ? "L2-warm" : "cold   ", name, NL, kb, mi, mt,
         kb * 1024 / (mt * 1e3));
  return 0;
}

int main() {
  char* src;
  float *big, *out;
  unsigned long long* st;
  const size_t nsrc = (size_t)256 << 20, nbig = (size_t)512 << 20;
  CK(hipMalloc(&src, nsrc)); CK(hipMemset(src, 0, nsrc));
  CK(hipMalloc(&big, nbig)); CK(hipMalloc(&out, 4096)); CK(hipMalloc(&st, 256 * 4 * 8));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t nf = nbig / 4;
#define RUN(NL, PAT, NAME) if (run<NL, PAT>(NAME, src, big, nf, st, out, s, warm)) return 1;
  for (int warm = 0; warm < 2; ++warm) {
    RUN(4, 0, "coalesced") RUN(10, 0, "coalesced") RUN(20, 0, "coalesced") RUN(40, 0, "coalesced")
    RUN(4, 1, "stride320") RUN(10, 1, "stride320") RUN(20, 1, "stride320") RUN(40, 1, "stride320")
    RUN(4, 2, "same") RUN(10, 2, "same") RUN(20, 2, "same") RUN(40, 2, "same")
  }
  printf("MB_OK\n");
  return 0;
}
