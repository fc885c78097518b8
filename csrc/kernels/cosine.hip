// Embedding-similarity scorers for the router (semantic-centroid strategy + semantic cache).
//   cosine_scores       : S[b, n] = <q_b, c_n> / (|q_b| |c_n|)      one wave per (b, n)
//   cache_scan          : a routing batch's semantic-cache lookups over the HBM table, one launch
//                         (context-id filter, then only the matching rows are read and scored)
//   cache_write         : a batch of deferred table row writes / removals, one launch
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

// ---- routing-cache scorer over the HBM table (reference: the per-entry Python loop of
// src/cache.py:267-305, restricted to entries of the query's context_key :280-293).
//
// One launch scores a whole routing batch (<= CQ queries): the table is [N, d] f32 rows with one
// int32 context id per row.  A lookup touches only the rows of its own context: every wave reads
// the context ids as 16-B vectors (4 rows per lane, 256 rows per wave-iteration: 4 B per row, 0.26 %
// of a 384-d row's bytes), matches them against the batch's sorted context ids (binary search in
// LDS), and only a matching row is fetched (16-B vector loads) and scored against the queries of
// its context (the row's norm is computed from the same registers: no norm table, no per-insert
// norm launch).  A hit is folded into best[q] with one 64-bit atomicMax of the orderable
// (sim << 32 | ~row) key: highest cosine wins, ties go to the lowest row, as numpy's argmax over
// slot order.  The batch descriptor (query addresses, sorted unique ids, groups) travels as a
// kernel argument, so a lookup is one launch plus the host read-back of best[] - no H2D copy.
constexpr int CQ = 128;
struct CacheScan {
  unsigned long long q[CQ];  // device address of query i's f32 [d] vector
  int ucid[CQ];              // sorted unique context ids of the batch
  int gbeg[CQ + 1];          // context u's queries: gq[gbeg[u] .. gbeg[u + 1])
  int gq[CQ];
  int nu;
};

template <int NV>  // float4 per lane per row: d / 4 <= 64 NV
__global__ void __launch_bounds__(256) cache_scan_kernel(CacheScan b, const float* __restrict__ table,
                                                         const int* __restrict__ ctx, long N, int d, float thr,
                                                         unsigned long long* __restrict__ best) {
  __shared__ int s_ucid[CQ], s_gbeg[CQ + 1], s_gq[CQ];
  __shared__ unsigned long long s_q[CQ];
  for (int i = threadIdx.x; i < CQ; i += blockDim.x) {
    s_ucid[i] = b.ucid[i];
    s_gq[i] = b.gq[i];
    s_q[i] = b.q[i];
  }
  for (int i = threadIdx.x; i <= CQ; i += blockDim.x) s_gbeg[i] = b.gbeg[i];
  __syncthreads();
  const int nu = b.nu, nf4 = d >> 2, lane = threadIdx.x & 63;
  const long nwave = (long)gridDim.x * (blockDim.x >> 6);
  // the next iteration's context ids are requested before this iteration's matches are scored, so
  // a wave that finds a match does not serialise its id stream behind the row fetch
  auto load_ids = [&](long r0, int (&c)[4]) {
    const long rb = r0 + 4 * lane;
    if (rb + 3 < N) {
      const int4 v = *reinterpret_cast<const int4*>(ctx + rb);
      c[0] = v.x; c[1] = v.y; c[2] = v.z; c[3] = v.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) c[k] = rb + k < N ? ctx[rb + k] : -1;
    }
  };
  long r0 = ((long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 256;
  int cn[4];
  if (r0 < N) load_ids(r0, cn);
  for (; r0 < N; r0 += nwave * 256) {
    int c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = cn[k];
    if (r0 + nwave * 256 < N) load_ids(r0 + nwave * 256, cn);
    int u[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int lo = 0, hi = nu;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_ucid[mid] < c[k]) lo = mid + 1; else hi = mid;
      }
      u[k] = (c[k] >= 0 && lo < nu && s_ucid[lo] == c[k]) ? lo : -1;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      unsigned long long m = __ballot(u[k] >= 0);
      while (m) {  // wave-uniform: one matching row at a time
        const int l = __builtin_ctzll(m);
        m &= m - 1;
        const long row = r0 + 4 * l + k;
        const int uu = __shfl(u[k], l, 64);
        const float4* rp = reinterpret_cast<const float4*>(table + row * d);
        float4 x[NV];
        float rr = 0.f;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const int i = lane + 64 * j;
          x[j] = i < nf4 ? rp[i] : make_float4(0.f, 0.f, 0.f, 0.f);
          rr += x[j].x * x[j].x + x[j].y * x[j].y + x[j].z * x[j].z + x[j].w * x[j].w;
        }
        rr = wave_sum(rr);
        const float nr = sqrtf(rr);
        for (int g = s_gbeg[uu]; g < s_gbeg[uu + 1]; ++g) {
          const int qi = s_gq[g];
          const float4* qp = reinterpret_cast<const float4*>(s_q[qi]);
          float dot = 0.f, qq = 0.f;
#pragma unroll
          for (int j = 0; j < NV; ++j) {
            const int i = lane + 64 * j;
            if (i < nf4) {
              const float4 y = qp[i];
              dot += x[j].x * y.x + x[j].y * y.y + x[j].z * y.z + x[j].w * y.w;
              qq += y.x * y.x + y.y * y.y + y.z * y.z + y.w * y.w;
            }
          }
          dot = wave_sum(dot);
          qq = wave_sum(qq);
          const float nq = sqrtf(qq);
          if (lane == 0 && nr >= 1e-9f && nq >= 1e-9f) {
            const float sim = dot / (nq * nr);
            if (sim >= thr)
              atomicMax(best + qi, ((unsigned long long)orderable(sim) << 32) | (0xffffffffu - (uint32_t)row));
          }
        }
      }
    }
  }
}

// Deferred table writes of a batch of inserts / removals (<= CW per launch, one workgroup each):
// row `slot` <- the f32 [d] vector at src (src 0: the row keeps its bytes), ctx[slot] <- cid
// (-1 removes the row from every lookup).  Replaces a copy launch plus a norm reduction per insert.
constexpr int CW = 64;
struct CacheWrite {
  unsigned long long src[CW];
  long long slot[CW];
  int cid[CW];
};

__global__ void __launch_bounds__(64) cache_write_kernel(CacheWrite w, float* __restrict__ table, int* __restrict__ ctx,
                                                         int d) {
  const int e = blockIdx.x;
  const long long slot = w.slot[e];
  const float4* src = reinterpret_cast<const float4*>(w.src[e]);
  if (src != nullptr) {
    float4* dst = reinterpret_cast<float4*>(table + slot * d);
    for (int i = threadIdx.x; i < (d >> 2); i += 64) dst[i] = src[i];
  }
  if (threadIdx.x == 0) ctx[slot] = w.cid[e];
}
}  // namespace

extern "C" int dllm_cosine_scores(const float* q, const float* c, float* s, int B, int N, int d, hipStream_t stream) {
  const long waves = (long)B * N;
  if (waves == 0) return 0;
  const long blocks = (waves * 64 + 255) / 256;
  hipLaunchKernelGGL(cosine_scores_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, q, c, s, B, N, d);
  return (int)hipGetLastError();
}

// qptr/qcid: nq <= CQ queries (device f32 [d] vectors and their context ids); best[nq] is zeroed here
extern "C" int dllm_cache_scan(const unsigned long long* qptr, const int* qcid, int nq, const float* table,
                               const int* ctx, long N, int d, float thr, unsigned long long* best, hipStream_t stream) {
  if (nq < 1 || nq > CQ || d % 4 || d > 64 * 4 * 4) return -22;
  const hipError_t e = hipMemsetAsync(best, 0, sizeof(unsigned long long) * nq, stream);
  if (e != hipSuccess) return (int)e;
  if (N <= 0) return 0;
  CacheScan b;
  // group the queries by context id (sorted unique ids, stable query order inside a group)
  int order[CQ];
  for (int i = 0; i < nq; ++i) order[i] = i;
  for (int i = 1; i < nq; ++i) {  // insertion sort by (cid, index): nq <= 128
    const int v = order[i];
    int j = i - 1;
    while (j >= 0 && qcid[order[j]] > qcid[v]) { order[j + 1] = order[j]; --j; }
    order[j + 1] = v;
  }
  int nu = 0;
  for (int i = 0; i < nq; ++i) {
    const int c = qcid[order[i]];
    if (nu == 0 || b.ucid[nu - 1] != c) { b.ucid[nu] = c; b.gbeg[nu] = i; ++nu; }
    b.gq[i] = order[i];
  }
  b.gbeg[nu] = nq;
  for (int i = nu; i < CQ; ++i) b.ucid[i] = 0x7fffffff;
  for (int i = nu + 1; i <= CQ; ++i) b.gbeg[i] = nq;
  for (int i = nq; i < CQ; ++i) b.gq[i] = 0;
  for (int i = 0; i < CQ; ++i) b.q[i] = i < nq ? qptr[i] : 0ull;
  b.nu = nu;
  long blocks = (N + 1023) / 1024;  // 4 waves x 256 rows per block-iteration
  if (blocks > 2048) blocks = 2048;  // 8 workgroups per CU; grid-stride over the rest
  const int nv = (d / 4 + 63) / 64;
  if (nv <= 1)
    hipLaunchKernelGGL(cache_scan_kernel<1>, dim3((unsigned)blocks), dim3(256), 0, stream, b, table, ctx, N, d, thr, best);
  else if (nv == 2)
    hipLaunchKernelGGL(cache_scan_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, stream, b, table, ctx, N, d, thr, best);
  else
    hipLaunchKernelGGL(cache_scan_kernel<4>, dim3((unsigned)blocks), dim3(256), 0, stream, b, table, ctx, N, d, thr, best);
  return (int)hipGetLastError();
}

extern "C" int dllm_cache_write(const unsigned long long* src, const long long* slot, const int* cid, int n, float* table,
                                int* ctx, int d, hipStream_t stream) {
  if (n < 0 || n > CW || d % 4) return -22;
  if (n == 0) return 0;
  CacheWrite w;
  for (int i = 0; i < CW; ++i) {
    w.src[i] = i < n ? src[i] : 0ull;
    w.slot[i] = i < n ? slot[i] : 0;
    w.cid[i] = i < n ? cid[i] : -1;
  }
  hipLaunchKernelGGL(cache_write_kernel, dim3(n), dim3(64), 0, stream, w, table, ctx, d);
  return (int)hipGetLastError();
}
