// Where the first microseconds of a dependent launch go (round-5 probe for the deep-level
// prologue): a hipGraph chain of kernels shaped like the conv launches (a 400-byte argument
// struct, 256 workgroups of 512 threads), each stamping s_memrealtime (100 MHz) at entry, once
// its first kernel argument is in an SGPR, once a first global load of a buffer the previous
// kernel wrote has returned, and at exit.  Variants:
//   0  arguments by value in the kernarg segment (what the runtime does today)
//   1  a pointer to the arguments in device memory (the struct read by s_load from HBM / L2)
//   2  the same, plus a 64-bit pointer argument only (kernarg preload candidate)
//   hipcc -O3 --offload-arch=gfx950 tools/mb_kernarg.hip -o tools/_mb_kernarg && ./tools/_mb_kernarg
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct Big {
  const float* in; float* out; int n; int k; long pad[46];
};
__device__ unsigned long long* g_st;   // [launch][block][4], not a kernel argument

__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void body(const Big& a, int launch, unsigned long long t0) {
  // t1: the first argument is available (the compiler waits for its s_load here)
  int n = a.n;
  asm volatile("" : "+s"(n));
  const unsigned long long t1 = rt();
  // t2: a global load of the previous kernel's output has returned
  float v = a.in[(blockIdx.x * blockDim.x + threadIdx.x) % n];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t2 = rt();
  a.out[(blockIdx.x * blockDim.x + threadIdx.x) % n] = v + 1.f;
  if (threadIdx.x == 0) {
    unsigned long long* s = g_st + ((size_t)launch * gridDim.x + blockIdx.x) * 4;
    s[0] = t0; s[1] = t1; s[2] = t2; s[3] = rt();
  }
}

__global__ __launch_bounds__(512) void k_byval(Big a, int launch) {
  const unsigned long long t0 = rt();
  body(a, launch, t0);
}
__global__ __launch_bounds__(512) void k_byptr(const Big* __restrict__ pa, int launch) {
  const unsigned long long t0 = rt();
  body(*pa, launch, t0);
}

int main() {
  const int L = 40, G = 256, NT = 512, n = 1 << 20;
  float *buf0, *buf1;
  CK(hipMalloc(&buf0, n * 4)); CK(hipMalloc(&buf1, n * 4));
  CK(hipMemset(buf0, 0, n * 4)); CK(hipMemset(buf1, 0, n * 4));
  unsigned long long* st;
  CK(hipMalloc(&st, sizeof(unsigned long long) * L * G * 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_st), &st, sizeof(st)));
  Big args[2];
  args[0] = Big{buf0, buf1, n, 0, {}};
  args[1] = Big{buf1, buf0, n, 0, {}};
  Big* dargs;
  CK(hipMalloc(&dargs, sizeof(Big) * 2));
  CK(hipMemcpy(dargs, args, sizeof(Big) * 2, hipMemcpyHostToDevice));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const char* names[2] = {"args by value (kernarg segment)", "args by pointer (device memory)"};
  for (int var = 0; var < 2; ++var) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int l = 0; l < L; ++l) {
      if (var == 0) hipLaunchKernelGGL(k_byval, dim3(G), dim3(NT), 0, s, args[l & 1], l);
      else hipLaunchKernelGGL(k_byptr, dim3(G), dim3(NT), 0, s, dargs + (l & 1), l);
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 20; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h((size_t)L * G * 4);
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    double d01 = 0, d12 = 0, d23 = 0, gap = 0, dur = 0;
    int ng = 0, nd = 0;
    for (int l = 2; l < L; ++l) {
      unsigned long long pmax = 0, cmin = ~0ull, cmax = 0;
      for (int b = 0; b < G; ++b) {
        const unsigned long long* p = &h[((size_t)(l - 1) * G + b) * 4];
        const unsigned long long* c = &h[((size_t)l * G + b) * 4];
        pmax = std::max(pmax, p[3]);
        cmin = std::min(cmin, c[0]);
        cmax = std::max(cmax, c[3]);
        d01 += c[1] - c[0]; d12 += c[2] - c[1]; d23 += c[3] - c[2];
        ++nd;
      }
      gap += (double)cmin - (double)pmax; dur += (double)(cmax - cmin);
      ++ng;
    }
    printf("%-34s entry->arg %.2f us  arg->load %.2f us  load->exit %.2f us | kernel span %.2f us, "
           "gap prev-exit->entry %.2f us\n", names[var], d01 / nd * 1e-2, d12 / nd * 1e-2, d23 / nd * 1e-2,
           dur / ng * 1e-2, gap / ng * 1e-2);
    // wall time per launch
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < 50; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-34s wall per launch %.2f us\n", names[var], ms * 1e3 / (50 * L));
    CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  }
  printf("MB_OK\n");
  return 0;
}
