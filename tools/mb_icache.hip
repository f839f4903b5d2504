// Is a large straight-line prologue bound by instruction fetch?  (round-5 probe: the deep conv
// kernels spend 3-7 us between block start and "all loads issued" with almost no memory work.)
// A hipGraph chain of 256-workgroup launches whose body is N dependent-free VALU instructions
// (v_add_f32 v?, 4 bytes each) either straight-line (N * 4 bytes of code) or as a loop over a
// 64-instruction body; stamps s_memrealtime before and after the body.  Kernels cycle over K
// distinct code copies so that the instruction cache holds (K = 1) or does not hold (K = 8,
// 8 x 16 KB) the previous launch's code.
//   hipcc -O3 --offload-arch=gfx950 tools/mb_icache.hip -o tools/_mb_icache && ./tools/_mb_icache
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ unsigned long long* g_st;

template <int COPY, int NINS>
__global__ __launch_bounds__(512) void k_straight(int launch) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  float a = threadIdx.x, b = 1.f;
  asm volatile(".rept %3\n v_add_f32 %0, %0, %1\n .endr\n s_nop %2" : "+v"(a) : "v"(b), "i"(COPY), "i"(NINS));
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    unsigned long long* s = g_st + ((size_t)launch * gridDim.x + blockIdx.x) * 4;
    s[0] = t0; s[1] = t1; s[2] = (unsigned long long)a; s[3] = 0;
  }
}
template <int COPY, int NINS>
__global__ __launch_bounds__(512) void k_loop(int launch) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  float a = threadIdx.x, b = 1.f;
  for (int i = 0; i < NINS / 64; ++i)
    asm volatile(".rept 64\n v_add_f32 %0, %0, %1\n .endr\n s_nop %2" : "+v"(a) : "v"(b), "i"(COPY));
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    unsigned long long* s = g_st + ((size_t)launch * gridDim.x + blockIdx.x) * 4;
    s[0] = t0; s[1] = t1; s[2] = (unsigned long long)a; s[3] = 0;
  }
}

typedef void (*KFn)(int);

template <int NINS>
static int run(const char* name, bool straight, int K, hipStream_t s, unsigned long long* st) {
  KFn ks[8] = {
    straight ? k_straight<0, NINS> : k_loop<0, NINS>, straight ? k_straight<1, NINS> : k_loop<1, NINS>,
    straight ? k_straight<2, NINS> : k_loop<2, NINS>, straight ? k_straight<3, NINS> : k_loop<3, NINS>,
    straight ? k_straight<4, NINS> : k_loop<4, NINS>, straight ? k_straight<5, NINS> : k_loop<5, NINS>,
    straight ? k_straight<6, NINS> : k_loop<6, NINS>, straight ? k_straight<7, NINS> : k_loop<7, NINS>};
  const int L = 32, G = 256;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int l = 0; l < L; ++l) hipLaunchKernelGGL(ks[l % K], dim3(G), dim3(512), 0, s, l);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int r = 0; r < 10; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  std::vector<unsigned long long> h((size_t)L * G * 4);
  CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
  double d = 0, mx = 0;
  int n = 0;
  for (int l = 8; l < L; ++l)
    for (int b = 0; b < G; ++b) {
      const double v = (double)(h[((size_t)l * G + b) * 4 + 1] - h[((size_t)l * G + b) * 4]) * 1e-2;
      d += v; mx = std::max(mx, v); ++n;
    }
  printf("%-10s %5d instr (%6d B of code)  %d code copies: body %.2f us mean, %.2f max (%.1f ns per instr)\n",
         name, NINS, straight ? NINS * 4 : 256, K, d / n, mx, d / n * 1e3 / NINS);
  CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
  return 0;
}

int main() {
  unsigned long long* st;
  CK(hipMalloc(&st, sizeof(unsigned long long) * 32 * 256 * 4));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_st), &st, sizeof(st)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int K : {1, 8}) {
    if (run<1024>("straight", true, K, s, st)) return 1;
    if (run<4096>("straight", true, K, s, st)) return 1;
    if (run<1024>("loop", false, K, s, st)) return 1;
    if (run<4096>("loop", false, K, s, st)) return 1;
  }
  printf("MB_OK\n");
  return 0;
}
