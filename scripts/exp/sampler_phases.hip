// Where a batch-1 sampled sampler launch goes (round 4): cumulative phases of row_topk on one
// Gaussian bf16 row (V = 32000, k = 40), us per launch over 400 back-to-back launches.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/kernels scripts/exp/sampler_phases.hip
#include "../../csrc/kernels/sampling.hip"
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

namespace {
template <int STOP>
__global__ void __launch_bounds__(SR_THREADS) phases(const u16* __restrict__ l, int V, int k, int* out) {
  __shared__ SrShared sh;
  const int tid = threadIdx.x;
  const int nv = V >> 3;
  if (STOP == 0) { if (tid == 0) out[0] = 1; return; }
  if (STOP >= 4) {
    const int n = row_topk(l, V, k, sh);
    if (STOP == 4) { if (tid == 0) out[0] = n + sh.i_r[0]; return; }
    if (tid < 64) {
      const int pick = draw_rank(sh, min(k, n), 0.8f, 0.9f, 7u, 0u);
      if (tid == 0) out[0] = sh.i_r[max(pick, 0)];
    }
    return;
  }
  unsigned tmax = 0u;
  for_each_vec<SR_THREADS>(l, nv, tid, [&](const uint4 v, int) {
    const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) tmax = max(tmax, bf_key(e[j]));
  });
  sh.hist[tid] = tmax;
  if (tid == 0) { sh.s_n = 0; sh.s_lo = 0; }
  __syncthreads();
  if (STOP == 1) { if (tid == 0) out[0] = sh.hist[5]; return; }
  int r = 0;
  const uint4* h4 = reinterpret_cast<const uint4*>(sh.hist);
  for (int j8 = 0; j8 < SR_THREADS / 4; j8 += 8) {
    uint4 o[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) o[u] = h4[j8 + u];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = 4 * (j8 + u);
      r += (o[u].x > tmax || (o[u].x == tmax && j < tid)) ? 1 : 0;
      r += (o[u].y > tmax || (o[u].y == tmax && j + 1 < tid)) ? 1 : 0;
      r += (o[u].z > tmax || (o[u].z == tmax && j + 2 < tid)) ? 1 : 0;
      r += (o[u].w > tmax || (o[u].w == tmax && j + 3 < tid)) ? 1 : 0;
    }
  }
  if (r == k - 1) sh.s_lo = (int)tmax;
  __syncthreads();
  if (STOP == 2) { if (tid == 0) out[0] = sh.s_lo; return; }
  const unsigned t0 = (unsigned)sh.s_lo;
  for_each_vec<SR_THREADS>(l, nv, tid, [&](const uint4 v, int c) {
    const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned key = bf_key(e[j]);
      if (key >= t0 && key != 0u) {
        const int p = atomicAdd(&sh.s_n, 1);
        if (p < SR_CAP) sh.cand[p] = make_float2(key_f(key), __int_as_float(c * 8 + j));
      }
    }
  });
  __syncthreads();
  if (tid == 0) out[0] = sh.s_n;
}
}  // namespace

template <int S>
static float run(const u16* d, int V, int k, int* o) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 50; ++i) phases<S><<<1, SR_THREADS>>>(d, V, k, o);
  hipEventRecord(a);
  for (int i = 0; i < 400; ++i) phases<S><<<1, SR_THREADS>>>(d, V, k, o);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / 400;
}

int main() {
  const int V = 32000, k = 40;
  std::vector<u16> h(V);
  std::mt19937 g(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  for (auto& x : h) { float f = nd(g); unsigned u; std::memcpy(&u, &f, 4); x = (u16)(u >> 16); }
  u16* d;
  int* o;
  hipMalloc(&d, V * 2);
  hipMalloc(&o, 64);
  hipMemcpy(d, h.data(), V * 2, hipMemcpyHostToDevice);
  int ns = 0;
  phases<3><<<1, SR_THREADS>>>(d, V, k, o);
  hipMemcpy(&ns, o, 4, hipMemcpyDeviceToHost);
  printf("{\"candidates_fast_path\": %d}\n", ns);
  printf("{\"stop\": 0, \"what\": \"empty launch\", \"us\": %.2f}\n", run<0>(d, V, k, o));
  printf("{\"stop\": 1, \"what\": \"+ scan 1 (thread maxima)\", \"us\": %.2f}\n", run<1>(d, V, k, o));
  printf("{\"stop\": 2, \"what\": \"+ rank of thread maxima\", \"us\": %.2f}\n", run<2>(d, V, k, o));
  printf("{\"stop\": 3, \"what\": \"+ scan 2 (candidate append)\", \"us\": %.2f}\n", run<3>(d, V, k, o));
  printf("{\"stop\": 4, \"what\": \"row_topk (+ rank of candidates)\", \"us\": %.2f}\n", run<4>(d, V, k, o));
  printf("{\"stop\": 5, \"what\": \"+ draw\", \"us\": %.2f}\n", run<5>(d, V, k, o));
  return 0;
}
