// Embedding-similarity scorers for the router (semantic-centroid strategy + semantic cache).
//   cosine_scores       : S[b, n] = <q_b, c_n> / (|q_b| |c_n|)      one wave per (b, n)
//   masked_cosine_argmax: over an HBM-resident cache table [N, d] with per-row norms and
//                         context-key ids, the best row with cos >= thr among rows whose ctx
//                         id matches — one fused pass (mask, dot, normalise, threshold,
//                         arg-max), grid-stride waves, wave reduction, one 64-bit atomicMax per
//                         wave on a packed (orderable-sim << 32 | ~row) key.  Replaces the
//                         reference's per-entry Python loop (src/cache.py:280-293).
#include "common.h"

namespace {

__global__ void cosine_scores_kernel(const float* __restrict__ q, const float* __restrict__ c, float* __restrict__ s,
                                     int B, int N, int d) {
  const long w = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= (long)B * N) return;
  const int b = (int)(w / N), n = (int)(w % N);
  const float* qb = q + (long)b * d;
  const float* cn = c + (long)n * d;
  float dot = 0.f, qq = 0.f, cc = 0.f;
  for (int i = lane; i < d; i += 64) {
    const float x = qb[i], y = cn[i];
    dot += x * y; qq += x * x; cc += y * y;
  }
  dot = wave_sum(dot); qq = wave_sum(qq); cc = wave_sum(cc);
  if (lane == 0) {
    const float nq = sqrtf(qq), nc = sqrtf(cc);
    s[w] = (nq < 1e-9f || nc < 1e-9f) ? 0.f : dot / (nq * nc);
  }
}

static __device__ __forceinline__ uint32_t orderable(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ void __launch_bounds__(256) masked_argmax_kernel(const float* __restrict__ q, const float* __restrict__ table,
                                                            const float* __restrict__ norms, const int* __restrict__ ctx,
                                                            int N, int d, int cid, float thr,
                                                            unsigned long long* __restrict__ best) {
  const int lane = threadIdx.x & 63;
  const long wave0 = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * blockDim.x) >> 6;
  float qq = 0.f;
  for (int i = lane; i < d; i += 64) qq += q[i] * q[i];
  const float nq = sqrtf(wave_sum(qq));
  unsigned long long mine = 0ull;
  if (nq >= 1e-9f) {
    for (long r = wave0; r < N; r += nwaves) {
      if (ctx[r] != cid) continue;            // wave-uniform branch
      const float nr = norms[r];
      if (nr < 1e-9f) continue;
      const float* row = table + r * d;
      float dot = 0.f;
      for (int i = lane; i < d; i += 64) dot += q[i] * row[i];
      dot = wave_sum(dot);
      const float sim = dot / (nq * nr);
      if (sim >= thr) {
        const unsigned long long key = ((unsigned long long)orderable(sim) << 32) | (0xffffffffu - (uint32_t)r);
        if (key > mine) mine = key;
      }
    }
  }
  if (lane == 0 && mine) atomicMax(best, mine);
}
}  // namespace

extern "C" int dllm_cosine_scores(const float* q, const float* c, float* s, int B, int N, int d, hipStream_t stream) {
  const long waves = (long)B * N;
  if (waves == 0) return 0;
  const long blocks = (waves * 64 + 255) / 256;
  hipLaunchKernelGGL(cosine_scores_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, q, c, s, B, N, d);
  return (int)hipGetLastError();
}

extern "C" int dllm_masked_cosine_argmax(const float* q, const float* table, const float* norms, const int* ctx, int N,
                                         int d, int cid, float thr, unsigned long long* best, hipStream_t stream) {
  const hipError_t e = hipMemsetAsync(best, 0, sizeof(unsigned long long), stream);
  if (e != hipSuccess) return (int)e;
  if (N <= 0) return 0;
  long blocks = ((long)N * 64 + 255) / 256;
  if (blocks > 2048) blocks = 2048;  // ~8 waves per CU; grid-stride over the rest
  hipLaunchKernelGGL(masked_argmax_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, q, table, norms, ctx, N, d, cid,
                     thr, best);
  return (int)hipGetLastError();
}
