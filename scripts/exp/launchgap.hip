// Experiment: per-kernel overhead of back-to-back dependent launches on one stream, eager and
// inside a hipGraph (empty kernels of 1 / 256 / 2048 workgroups, and a 4 MB copy kernel).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/exp/bin/launchgap scripts/exp/launchgap.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_empty(int* p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1; }
__global__ void k_copy(const float4* a, float4* b, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) b[i] = a[i];
}

int main() {
  int* p;
  float4 *a, *b;
  const int n = (4 << 20) / 16;
  CHECK(hipMalloc(&p, 64)); CHECK(hipMemset(p, 0, 64));
  CHECK(hipMalloc(&a, n * 16)); CHECK(hipMalloc(&b, n * 16));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  const int N = 200;
  struct Cfg { const char* name; int grid; int copy; } cfgs[] = {{"empty_1wg", 1, 0}, {"empty_256wg", 256, 0},
                                                                 {"empty_2048wg", 2048, 0}, {"copy_4MB_1024wg", 1024, 1}};
  for (auto& c : cfgs) {
    auto launch = [&] {
      if (c.copy) hipLaunchKernelGGL(k_copy, dim3(c.grid), dim3(256), 0, s, a, b, n);
      else hipLaunchKernelGGL(k_empty, dim3(c.grid), dim3(256), 0, s, p);
    };
    for (int i = 0; i < 20; ++i) launch();
    CHECK(hipStreamSynchronize(s));
    CHECK(hipEventRecord(e0, s));
    for (int i = 0; i < N; ++i) launch();
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms_eager;
    CHECK(hipEventElapsedTime(&ms_eager, e0, e1));
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < N; ++i) launch();
    CHECK(hipStreamEndCapture(s, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHECK(hipGraphLaunch(ge, s));
    CHECK(hipStreamSynchronize(s));
    CHECK(hipEventRecord(e0, s));
    for (int r = 0; r < 5; ++r) CHECK(hipGraphLaunch(ge, s));
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms_graph;
    CHECK(hipEventElapsedTime(&ms_graph, e0, e1));
    printf("{\"exp\": \"launchgap\", \"kernel\": \"%s\", \"eager_us_per_kernel\": %.2f, \"graph_us_per_kernel\": %.2f}\n",
           c.name, ms_eager * 1000 / N, ms_graph * 1000 / (5 * N));
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
  }
  return 0;
}
