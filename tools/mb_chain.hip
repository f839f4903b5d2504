// Hand-off calibration for a persistent per-image layer chain (the UNet deep levels as one launch):
// NT teams of G workgroups (one team per image), L layers; in every layer each member waits until
// its team's counter shows all G members finished the previous layer, reads the team's previous
// output (sc0 sc1 loads, checking every word's tag), writes its slice of this layer's output
// (sc0 sc1 stores), drains (vmcnt(0)), barrier, one agent-scope atomic add.  Reported: µs per
// layer for the chain against the same L layers as L dependent launches of a graph, and the
// number of stale words read (must be 0).  Spins are bounded (s_memrealtime, 100 MHz): a stuck
// team sets an error word and leaves, it never hangs the device.
//   hipcc -O3 --offload-arch=gfx950 tools/mb_chain.hip -o tools/_mbc && ./tools/_mbc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) volatile u4 gvu4;   // global (not flat) sc0 sc1 accesses

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct P {
  unsigned* counter;     // [NT]
  unsigned* err;         // [1]
  unsigned* bad;         // [1] stale words seen
  u4* buf;            // [L + 1][NT][IN / 16]
  int NT, G, L, in_bytes, spread, work;
};

__device__ __forceinline__ bool wait_count(const P& p, unsigned* c, unsigned target) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {   // 200 ms
        __hip_atomic_store(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  return __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
}

__global__ __launch_bounds__(512) void k_chain(P p) {
  const int team = p.spread ? blockIdx.x / p.G : blockIdx.x % p.NT;
  const int mem = p.spread ? blockIdx.x % p.G : blockIdx.x / p.NT;
  const int nu = p.in_bytes / 16;                 // 16-byte units of one team's layer output
  const int per = nu / p.G;                       // units each member writes
  unsigned stale = 0;
  float acc = 0.f;
  for (int l = 1; l <= p.L; ++l) {
    if (!wait_count(p, p.counter + team, (unsigned)(p.G * (l - 1)))) return;
    const gvu4* in = (const gvu4*)(p.buf + ((size_t)(l - 1) * p.NT + team) * nu);
    for (int u = threadIdx.x; u < nu; u += blockDim.x) {
      const u4 v = in[u];
      if (l > 1 && (v.x != (unsigned)(l - 1) || v.y != (unsigned)team || v.z != (unsigned)u)) ++stale;
      acc += __uint_as_float(v.w & 0x3fffffffu);
    }
    for (int k = 0; k < p.work; ++k) acc = acc * 0.999f + 1e-3f;
    gvu4* out = (gvu4*)(p.buf + ((size_t)l * p.NT + team) * nu);
    for (int u = mem * per + threadIdx.x; u < (mem + 1) * per; u += blockDim.x)
      out[u] = u4{(unsigned)l, (unsigned)team, (unsigned)u, __float_as_uint(acc) & 0x3fffffffu};
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(p.counter + team, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (stale) atomicAdd(p.bad, stale);
}

// one layer as its own launch (the launch-chain baseline): read the team's previous output, write a slice
__global__ __launch_bounds__(512) void k_layer(P p, int l) {
  const int team = blockIdx.x / p.G, mem = blockIdx.x % p.G;
  const int nu = p.in_bytes / 16, per = nu / p.G;
  const u4* in = p.buf + ((size_t)(l - 1) * p.NT + team) * nu;
  float acc = 0.f;
  for (int u = threadIdx.x; u < nu; u += blockDim.x) acc += __uint_as_float(in[u].w & 0x3fffffffu);
  for (int k = 0; k < p.work; ++k) acc = acc * 0.999f + 1e-3f;
  u4* out = p.buf + ((size_t)l * p.NT + team) * nu;
  for (int u = mem * per + threadIdx.x; u < (mem + 1) * per; u += blockDim.x)
    out[u] = u4{(unsigned)l, (unsigned)team, (unsigned)u, __float_as_uint(acc) & 0x3fffffffu};
}

int main() {
  const int NT = 16, G = 16, L = 20;
  P p{};
  p.NT = NT; p.G = G; p.L = L;
  const int max_in = 131072;
  CK(hipMalloc(&p.counter, sizeof(unsigned) * NT));
  CK(hipMalloc(&p.err, 4));
  CK(hipMalloc(&p.bad, 4));
  CK(hipMalloc(&p.buf, (size_t)(L + 1) * NT * max_in));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (int in_bytes : {8192, 40960, 131072}) {
    for (int work : {0, 2000}) {
      p.in_bytes = in_bytes; p.work = work;
      for (int spread : {0, 1}) {
        p.spread = spread;
        float best = 1e9f;
        unsigned err = 0, bad = 0;
        for (int rep = 0; rep < 6; ++rep) {
          CK(hipMemsetAsync(p.counter, 0, sizeof(unsigned) * NT, s));
          CK(hipMemsetAsync(p.err, 0, 4, s));
          CK(hipMemsetAsync(p.bad, 0, 4, s));
          CK(hipEventRecord(e0, s));
          hipLaunchKernelGGL(k_chain, dim3(NT * G), dim3(512), 0, s, p);
          CK(hipGetLastError());
          CK(hipEventRecord(e1, s));
          CK(hipStreamSynchronize(s));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          unsigned e = 0, b = 0;
          CK(hipMemcpy(&e, p.err, 4, hipMemcpyDeviceToHost));
          CK(hipMemcpy(&b, p.bad, 4, hipMemcpyDeviceToHost));
          err |= e; bad += b;
          if (rep > 0 && ms < best) best = ms;
        }
        printf("chain   in=%6d work=%4d %s: %7.2f us/layer  (err %u, stale words %u)\n", in_bytes, work,
               spread ? "team spread over XCDs" : "team on one XCD      ", best * 1e3f / L, err, bad);
      }
      // the same layers as dependent launches captured in a graph
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int l = 1; l <= L; ++l) hipLaunchKernelGGL(k_layer, dim3(NT * G), dim3(512), 0, s, p, l);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      float best = 1e9f;
      for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(e0, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s));
        CK(hipStreamSynchronize(s));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
      }
      printf("launches in=%6d work=%4d                      : %7.2f us/layer\n", in_bytes, work, best * 1e3f / L);
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  printf("MB_CHAIN_OK\n");
  return 0;
}
