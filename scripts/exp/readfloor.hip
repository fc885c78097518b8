// Experiment: time to stream an N-MB weight matrix once (no math) inside a hipGraph, rotating over
// 64 distinct buffers so every launch reads from HBM — the floor under a decode GEMM of that size.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/exp/bin/readfloor scripts/exp/readfloor.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void k_read(const uint4* __restrict__ a, long n16, unsigned* out) {
  unsigned acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  unsigned* out;
  CHECK(hipMalloc(&out, 64));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  for (long mb : {8L, 23L, 46L, 128L}) {
    const int copies = 64;
    std::vector<uint4*> bufs(copies);
    const long bytes = mb << 20;
    for (auto& b : bufs) { CHECK(hipMalloc(&b, bytes)); CHECK(hipMemset(b, 1, bytes)); }
    for (int grid : {256, 1024, 4096}) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int i = 0; i < copies; ++i) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, s, bufs[i], bytes / 16, out);
      CHECK(hipStreamEndCapture(s, &g));
      CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CHECK(hipGraphLaunch(ge, s));
      CHECK(hipStreamSynchronize(s));
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
      CHECK(hipEventRecord(e0, s));
      for (int r = 0; r < 5; ++r) CHECK(hipGraphLaunch(ge, s));
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1000 / (5 * copies);
      printf("{\"exp\": \"readfloor\", \"MB\": %ld, \"grid\": %d, \"us_per_read\": %.2f, \"TBps\": %.2f}\n", mb, grid, us,
             bytes / (us * 1e-6) / 1e12);
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(g));
    }
    for (auto& b : bufs) CHECK(hipFree(b));
  }
  return 0;
}
