// Latency calibration on the MI355X box: average duration of small kernels replayed in a
// hipGraph chain (the same launch structure as the sampler's step graph).
//   hipcc -O3 --offload-arch=gfx950 tools/microbench.hip -o tools/_mb && ./tools/_mb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_empty(float* p) {
  if (p == nullptr) p[threadIdx.x] = 0.f;
}
__global__ void k_load_store(const float* __restrict__ in, float* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  out[i % n] = in[i % n] + 1.f;
}
// dependent chain of `hops` loads per thread (pointer chase through an index array)
__global__ void k_chase(const int* __restrict__ idx, float* out, int hops, int n) {
  int j = (blockIdx.x * blockDim.x + threadIdx.x) % n;
  for (int h = 0; h < hops; ++h) j = idx[j];
  out[(blockIdx.x * blockDim.x + threadIdx.x) % n] = (float)j;
}
__global__ void k_spin(float* out, int iters) {
  float v = threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) v = v * 0.999f + 1e-3f;
  if (v == -1.f) out[0] = v;
}
__global__ void k_barriers(float* out, int nb) {
  __shared__ float s[256];
  float v = threadIdx.x;
  for (int i = 0; i < nb; ++i) {
    s[threadIdx.x] = v;
    __syncthreads();
    v += s[(threadIdx.x + 1) & 255];
    __syncthreads();
  }
  if (v == -1.f) out[0] = v;
}
__global__ void k_store_then_barrier(float* out, int n, int reps) {
  __shared__ float s[256];
  float v = threadIdx.x;
  for (int r = 0; r < reps; ++r) {
    out[((blockIdx.x * reps + r) * blockDim.x + threadIdx.x) % n] = v;
    s[threadIdx.x] = v;
    __syncthreads();
    v += s[(threadIdx.x + 1) & 255];
  }
}

template <typename F>
static float time_graph(hipStream_t s, int reps, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < reps; ++i) launch();
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, s);
  for (int k = 0; k < 5; ++k) hipGraphLaunch(ge, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return ms * 1000.f / (5 * reps);
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int n = 1 << 22;                 // 16 MB buffers
  float *in, *out;
  int* idx;
  CK(hipMalloc(&in, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&idx, n * 4));
  std::vector<int> h(n);
  for (int i = 0; i < n; ++i) h[i] = (int)(((long long)i * 2654435761LL + 12345) % n);
  CK(hipMemcpy(idx, h.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemset(in, 0, n * 4));
  const int R = 200;
  for (int blocks : {80, 256, 1024}) {
    printf("blocks %4d: empty %6.2f us", blocks, time_graph(s, R, [&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, s, out); }));
    printf(" | load+store(1MB) %6.2f", time_graph(s, R, [&] { hipLaunchKernelGGL(k_load_store, dim3(blocks), dim3(256), 0, s, in, out, 1 << 18); }));
    for (int hops : {1, 4, 16})
      printf(" | chase%-2d(16MB) %6.2f", hops, time_graph(s, R, [&] { hipLaunchKernelGGL(k_chase, dim3(blocks), dim3(256), 0, s, idx, out, hops, n); }));
    printf(" | 20 barriers %6.2f", time_graph(s, R, [&] { hipLaunchKernelGGL(k_barriers, dim3(blocks), dim3(256), 0, s, out, 10); }));
    printf(" | 8x(store+barrier) %6.2f\n", time_graph(s, R, [&] { hipLaunchKernelGGL(k_store_then_barrier, dim3(blocks), dim3(256), 0, s, out, n, 8); }));
  }
  {  // stream concurrency: two graphs (each R chase kernels of 80 blocks) on one vs two streams
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto mk = [&](hipStream_t st, hipGraphExec_t* ge) {
      hipGraph_t g;
      (void)hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
      for (int i = 0; i < R; ++i) hipLaunchKernelGGL(k_spin, dim3(80), dim3(256), 0, st, out, 4000);
      (void)hipStreamEndCapture(st, &g);
      (void)hipGraphInstantiate(ge, g, nullptr, nullptr, 0);
    };
    hipGraphExec_t g1, g2;
    mk(s, &g1);
    mk(s2, &g2);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int mode = 0; mode < 2; ++mode) {
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, s);
      (void)hipStreamWaitEvent(s2, e0, 0);
      for (int k = 0; k < 3; ++k) {
        (void)hipGraphLaunch(g1, s);
        (void)hipGraphLaunch(g2, mode ? s2 : s);
      }
      hipEvent_t e2;
      (void)hipEventCreate(&e2);
      (void)hipEventRecord(e2, s2);
      (void)hipStreamWaitEvent(s, e2, 0);
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("two graphs of %d spin kernels x3 on %s: %.1f us per kernel pair\n", R, mode ? "two streams" : "one stream", ms * 1000.f / (3 * R));
    }
  }
  {  // (a) eager launches alternating on two streams; (b) one graph with two parallel branches
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e0, e1, e2;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); (void)hipEventCreate(&e2);
    for (int mode = 0; mode < 2; ++mode) {
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, s);
      (void)hipStreamWaitEvent(s2, e0, 0);
      for (int i = 0; i < R; ++i) {
        hipLaunchKernelGGL(k_spin, dim3(80), dim3(256), 0, s, out, 4000);
        hipLaunchKernelGGL(k_spin, dim3(80), dim3(256), 0, mode ? s2 : s, out, 4000);
      }
      (void)hipEventRecord(e2, s2);
      (void)hipStreamWaitEvent(s, e2, 0);
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("eager pairs of spin kernels on %s: %.1f us per pair\n", mode ? "two streams" : "one stream", ms * 1000.f / R);
    }
    // one graph, two branches forked from s
    hipGraph_t g;
    hipGraphExec_t ge;
    hipEvent_t ef, ej;
    (void)hipEventCreateWithFlags(&ef, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&ej, hipEventDisableTiming);
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    (void)hipEventRecord(ef, s);
    (void)hipStreamWaitEvent(s2, ef, 0);
    for (int i = 0; i < R; ++i) {
      hipLaunchKernelGGL(k_spin, dim3(80), dim3(256), 0, s, out, 4000);
      hipLaunchKernelGGL(k_spin, dim3(80), dim3(256), 0, s2, out, 4000);
    }
    (void)hipEventRecord(ej, s2);
    (void)hipStreamWaitEvent(s, ej, 0);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    (void)hipGraphLaunch(ge, s);
    (void)hipStreamSynchronize(s);
    (void)hipEventRecord(e0, s);
    for (int k = 0; k < 3; ++k) (void)hipGraphLaunch(ge, s);
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("one graph with two parallel branches: %.1f us per pair\n", ms * 1000.f / (3 * R));
  }
  int lds_kb = 128;
  printf("empty kernel with %d KB dynamic LDS, 256 blocks: %6.2f us\n", lds_kb,
         time_graph(s, R, [&] { hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), lds_kb * 1024, s, out); }));
  return 0;
}
