// Token sampling on the logits of the last position of every sequence.
//   argmax_kernel      : greedy (temperature 0) — one workgroup per row, 16-B loads of bf16/f32
//                        logits, wave-shuffle arg-max (ties -> lowest index, like torch.argmax).
//   sample_topp_kernel : temperature + top-p (nucleus) sampling over the row's top-K candidates
//                        (values sorted descending, from a top-k pass), one wave per row,
//                        inverse-CDF draw with a per-row uniform u in [0,1).
//   sample_rows_kernel : the whole sampler for one decode step in ONE launch (graph-captured):
//                        per row, greedy -> arg-max, else exact top-k of the bf16 logits, then
//                        temperature, nucleus cut and inverse-CDF draw — no torch.topk kernel
//                        chain, no second LM-head GEMM, no host round trip for sampled rows.
#include "common.h"

namespace {

static __device__ __forceinline__ void better(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
}

template <bool BF16>
__global__ void __launch_bounds__(256) argmax_kernel(const void* __restrict__ logits, long stride, int V,
                                                     int* __restrict__ out) {
  __shared__ float sv[8];
  __shared__ int si[8];
  const int row = blockIdx.x;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  if (BF16) {
    const u16* l = reinterpret_cast<const u16*>(logits) + row * stride;
    const int nv = V >> 3;
    for (int c = threadIdx.x; c < nv; c += blockDim.x) {
      float f[8];
      unpack8(ld16(l + c * 8), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) better(bv, bi, f[j], c * 8 + j);
    }
    for (int i = (nv << 3) + threadIdx.x; i < V; i += blockDim.x) better(bv, bi, bf2f(l[i]), i);
  } else {
    const float* l = reinterpret_cast<const float*>(logits) + row * stride;
    const int nv = V >> 2;
    for (int c = threadIdx.x; c < nv; c += blockDim.x) {
      float4 f = reinterpret_cast<const float4*>(l)[c];
      better(bv, bi, f.x, 4 * c); better(bv, bi, f.y, 4 * c + 1);
      better(bv, bi, f.z, 4 * c + 2); better(bv, bi, f.w, 4 * c + 3);
    }
    for (int i = (nv << 2) + threadIdx.x; i < V; i += blockDim.x) better(bv, bi, l[i], i);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(bv, o, 64);
    int oi = __shfl_xor(bi, o, 64);
    better(bv, bi, ov, oi);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sv[wid] = bv; si[wid] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) better(bv, bi, sv[w], si[w]);
    out[row] = (bi == 0x7fffffff) ? 0 : bi;
  }
}

// vals [B, K] sorted desc (f32), idx [B, K] int64; temp/top_p/u per row
__global__ void sample_topp_kernel(const float* __restrict__ vals, const long* __restrict__ idx, int K,
                                   const float* __restrict__ temp, const float* __restrict__ top_p,
                                   const float* __restrict__ u, int* __restrict__ out) {
  const int row = blockIdx.x, lane = threadIdx.x;
  const float* v = vals + (long)row * K;
  const float t = fmaxf(temp[row], 1e-5f);
  const float m = v[0];
  // total mass over candidates
  float s = 0.f;
  for (int i = lane; i < K; i += 64) s += __expf((v[i] - m) / t);
  s = wave_sum(s);
  // nucleus cut: smallest prefix with cumulative prob >= top_p (serial over the sorted list)
  if (lane == 0) {
    const float tp = top_p[row];
    float c = 0.f;
    int n = K;
    for (int i = 0; i < K; ++i) {
      c += __expf((v[i] - m) / t) / s;
      if (c >= tp) { n = i + 1; break; }
    }
    float mass = 0.f;
    for (int i = 0; i < n; ++i) mass += __expf((v[i] - m) / t);
    const float target = u[row] * mass;
    float acc = 0.f;
    int pick = n - 1;
    for (int i = 0; i < n; ++i) {
      acc += __expf((v[i] - m) / t);
      if (acc > target) { pick = i; break; }
    }
    out[row] = (int)idx[(long)row * K + pick];
  }
}
// ---------------------------------------------------------------------------- fused row sampler
// Exact top-k (k <= 256) without sorting 32 K logits:
//   1. histogram of the 12 high bits of a monotonic 16-bit key of each bf16 logit (LDS atomics;
//      3 mantissa bits per bin keep same-address conflicts low), a block-wide scan from the top
//      finds the bin holding the k-th largest; if that bin is crowded (> SR_MAXN candidates) a
//      second 16-bin pass over its low 4 bits pins the exact threshold key;
//   2. every logit at or above the threshold is appended to an LDS candidate list;
//   3. rank of each candidate = #candidates strictly better (value desc, index asc: the same tie
//      rule as torch.argmax), an O(n^2) LDS-broadcast pass — no sort; ranks < k are the top-k,
//      written in rank order;
//   4. wave 0: softmax weights at temperature t, inclusive prefix sums in rank order (wave scan),
//      nucleus = shortest prefix with mass >= top_p, inverse-CDF pick with u = hash(seed, row).
constexpr int SR_THREADS = 256;
constexpr int SR_CAP = 1024;   // candidate list capacity (only ties AT the threshold key can be dropped)
constexpr int SR_MAXN = 512;   // above this many candidates the exact-threshold pass runs
constexpr int SR_KMAX = 256;

// Visit a row's 16-B logit vectors c = tid, tid + NT, ... four at a time with all four loads
// issued before the first is used (a row is ~16 vectors per thread: one dependent round trip per
// vector was most of a batch-1 sampler launch).  f(vec, c) sees every vector exactly once.
template <int NT, class F>
static __device__ __forceinline__ void for_each_vec(const u16* __restrict__ l, int nv, int tid, F f) {
  int c = tid;
  for (; c + 3 * NT < nv; c += 4 * NT) {
    const uint4 v0 = ld16(l + (long)c * 8), v1 = ld16(l + (long)(c + NT) * 8);
    const uint4 v2 = ld16(l + (long)(c + 2 * NT) * 8), v3 = ld16(l + (long)(c + 3 * NT) * 8);
    f(v0, c);
    f(v1, c + NT);
    f(v2, c + 2 * NT);
    f(v3, c + 3 * NT);
  }
  for (; c < nv; c += NT) f(ld16(l + (long)c * 8), c);
}

static __device__ __forceinline__ unsigned bf_key(u16 b) {
  if ((b & 0x7f80) == 0x7f80 && (b & 0x7f)) return 0u;  // NaN: never selected
  return (b & 0x8000) ? (unsigned)(~b & 0xffff) : (unsigned)(b | 0x8000);
}

static __device__ __forceinline__ float key_f(unsigned k) {
  return bf2f((k & 0x8000) ? (u16)(k & 0x7fff) : (u16)(~k & 0xffff));
}

// counter-based uniform in [0, 1): identical on host (ops.reference.row_uniform)
static __device__ __forceinline__ float row_uniform(unsigned seed, unsigned row) {
  unsigned h = seed + row * 0x9E3779B9u;
  h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
  return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// Shared state of one row's selection (one workgroup per row).
struct SrShared {
  alignas(16) unsigned hist[4096];
  alignas(16) float2 cand[SR_CAP];   // (value, index bits)
  float w_r[SR_KMAX];           // value by rank
  int i_r[SR_KMAX];             // token id by rank
  unsigned wsum[SR_THREADS / 64];
  float sv[SR_THREADS / 64];
  int si[SR_THREADS / 64];
  int s_bin, s_above, s_n, s_nt, s_lo, s_amax;
  float s_m;
};

// Phases 0-3 over one row of V bf16 logits: afterwards sh.w_r / sh.i_r hold the exact top
// min(k, n) (value desc, index asc) and sh.s_m the row maximum; returns n (every thread), the
// candidate count, which is < k only for rows with fewer than k non-NaN logits.
static __device__ __forceinline__ int row_topk(const u16* __restrict__ l, int V, int k, SrShared& sh) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nv = V >> 3;
  // ---- 0. fast bound (no histogram): T0 from the 256 per-thread maximum keys (below) such that
  // at least k logits are >= T0, so every top-k logit is too;
  // when few logits reach T0 (typical: ~k-3k of 32 K) they are the whole candidate list and the
  // 4096-bin LDS-atomic histogram (hot bins serialise its atomics: ~40 us for one row) is skipped.
  // A flat row (> SR_MAXN logits at or above T0) falls through to the histogram path.
  {
    // rows of <= 32K logits (16 vectors per thread) are loaded ONCE, all 16 loads in flight, and
    // both scans below read the registers; longer rows stream twice (for_each_vec)
    constexpr int RC = 16;
    uint4 cv[RC];
    const bool cached = nv <= RC * SR_THREADS;
    if (cached) {
#pragma unroll
      for (int u = 0; u < RC; ++u) {
        const int c = tid + u * SR_THREADS;
        cv[u] = c < nv ? ld16(l + (long)c * 8) : make_uint4(0u, 0u, 0u, 0u);
      }
    }
    auto visit = [&](auto f) {
      if (cached) {
#pragma unroll
        for (int u = 0; u < RC; ++u) {
          const int c = tid + u * SR_THREADS;
          if (c < nv) f(cv[u], c);
        }
      } else {
        for_each_vec<SR_THREADS>(l, nv, tid, f);
      }
    };
    unsigned tmax = 0u;
    visit([&](const uint4 v, int) {
      const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) tmax = max(tmax, bf_key(e[j]));
    });
    for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) tmax = max(tmax, bf_key(l[i]));
    if (tid == 0) sh.s_n = 0;
    // T0 = the smallest of the 4 waves' ceil(k/4)-th largest thread maximum: every wave has at
    // least ceil(k/4) threads whose maximum is >= T0, so at least k logits are.  Per wave: each
    // lane counts the wave's maxima above its own (uniform lane reads, no LDS); the lane of rank
    // ceil(k/4) - 1 (ties -> lower lane) publishes.  (An exact k-th of all 256 maxima through LDS
    // was ~5 us of a ~27 us batch-1 launch, profiles/r4_sampler.md.)
    const int kw = (k + 3) >> 2;
    int r = 0;
    for (int j = 0; j < 64; ++j) {
      const unsigned o = (unsigned)__builtin_amdgcn_readlane((int)tmax, j);
      r += (o > tmax || (o == tmax && j < lane)) ? 1 : 0;
    }
    if (r == kw - 1) sh.wsum[wid] = tmax;
    __syncthreads();
    if (tid == 0) {
      unsigned t = sh.wsum[0];
      for (int w = 1; w < SR_THREADS / 64; ++w) t = min(t, sh.wsum[w]);
      sh.s_lo = (int)t;
    }
    __syncthreads();
    const unsigned t0 = (unsigned)sh.s_lo;
    // candidates are rare (~k-3k of 32K): a branch-free 8-bit mask per vector, and the appends
    // (LDS atomics) only for set bits -- one branch per vector instead of one per logit (the
    // per-logit form was ~12 us of the batch-1 launch)
    visit([&](const uint4 v, int c) {
      const u16* e = reinterpret_cast<const u16*>(&v);
      unsigned m = 0u;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned key = bf_key(e[j]);
        m |= (key >= t0 && key != 0u) ? (1u << j) : 0u;
      }
      while (m) {
        const int j = __builtin_ctz(m);
        m &= m - 1u;
        // element j without indexing the vector (a dynamic index would put it in scratch)
        const unsigned w = (j < 4) ? ((j < 2) ? v.x : v.y) : ((j < 6) ? v.z : v.w);
        const unsigned key = bf_key((u16)((j & 1) ? (w >> 16) : (w & 0xffffu)));
        const int p = atomicAdd(&sh.s_n, 1);
        if (p < SR_CAP) sh.cand[p] = make_float2(key_f(key), __int_as_float(c * 8 + j));
      }
    });
    for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) {
      const unsigned key = bf_key(l[i]);
      if (key >= t0 && key != 0u) {
        const int p = atomicAdd(&sh.s_n, 1);
        if (p < SR_CAP) sh.cand[p] = make_float2(key_f(key), __int_as_float(i));
      }
    }
    __syncthreads();
  }
  int na, nt;
  if (sh.s_n >= k && sh.s_n <= SR_MAXN) {
    na = sh.s_n;
    nt = 0;
  } else {
  __syncthreads();  // every thread has read s_n before the histogram path reuses it

  // ---- 1. coarse histogram (12-bit bins) and the bin of the k-th largest
  for (int i = tid; i < 4096; i += SR_THREADS) sh.hist[i] = 0u;
  if (tid == 0) { sh.s_bin = 0; sh.s_above = 0; }   // a row with < k non-NaN logits keeps them all
  __syncthreads();
  for (int c = tid; c < nv; c += SR_THREADS) {
    const uint4 v = ld16(l + c * 8);
    const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(&sh.hist[bf_key(e[j]) >> 4], 1u);
  }
  for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) atomicAdd(&sh.hist[bf_key(l[i]) >> 4], 1u);
  __syncthreads();
  unsigned mine = 0;  // thread t owns bins 4095-16t .. 4080-16t (descending key order)
#pragma unroll
  for (int j = 0; j < 16; ++j) mine += sh.hist[4095 - 16 * tid - j];
  unsigned x = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh.wsum[wid] = x;
  __syncthreads();
  unsigned base = 0;
  for (int w = 0; w < wid; ++w) base += sh.wsum[w];
  const unsigned incl = base + x, excl = incl - mine;
  if (excl < (unsigned)k && incl >= (unsigned)k) {  // exactly one thread
    unsigned acc = excl;
    for (int j = 0; j < 16; ++j) {
      const int b = 4095 - 16 * tid - j;
      if (acc + sh.hist[b] >= (unsigned)k) { sh.s_bin = b; sh.s_above = (int)acc; break; }
      acc += sh.hist[b];
    }
  }
  __syncthreads();
  const int bin = sh.s_bin;
  if (sh.s_above + (int)sh.hist[bin] > SR_MAXN) {  // crowded bin: exact threshold from its low 4 bits
    __syncthreads();
    if (tid < 16) sh.hist[tid] = 0u;            // hist[0..15] re-used as the 16 fine bins (the coarse
    __syncthreads();                            // counts are no longer needed past this point)
    for (int c = tid; c < nv; c += SR_THREADS) {
      const uint4 v = ld16(l + c * 8);
      const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned key = bf_key(e[j]);
        if ((int)(key >> 4) == bin) atomicAdd(&sh.hist[key & 15], 1u);
      }
    }
    for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) {
      const unsigned key = bf_key(l[i]);
      if ((int)(key >> 4) == bin) atomicAdd(&sh.hist[key & 15], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned acc = (unsigned)sh.s_above;
      int lo = bin << 4;
      for (int b = 15; b >= 0; --b) {
        if (acc + sh.hist[b] >= (unsigned)k) { lo = (bin << 4) | b; break; }
        acc += sh.hist[b];
      }
      sh.s_lo = lo;
      sh.s_amax = (int)acc;  // exactly the keys strictly above lo (< k)
    }
  } else if (tid == 0) {
    sh.s_lo = bin << 4;
    sh.s_amax = sh.s_above + (int)sh.hist[bin];  // every candidate (<= SR_MAXN): none is ever dropped
  }
  if (tid == 0) { sh.s_n = 0; sh.s_nt = 0; }
  __syncthreads();

  // ---- 2. candidates: every logit at or above the threshold key.  Keys strictly above it (at most
  // s_amax: < k for a crowded bin, <= SR_MAXN otherwise) fill slots from the bottom; ties AT the
  // threshold fill slots from the top, never below slot s_amax — so a crowded tie bin can only
  // drop ties, never a strictly better logit, and the top-k stays exact.  NaN (key 0) never enters.
  const unsigned lo = (unsigned)sh.s_lo;
  const int amax = min(sh.s_amax, SR_CAP);
  for (int c = tid; c < nv; c += SR_THREADS) {
    const uint4 v = ld16(l + c * 8);
    const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned key = bf_key(e[j]);
      if (key == 0u) continue;
      if (key > lo) {
        const int p = atomicAdd(&sh.s_n, 1);
        if (p < amax) sh.cand[p] = make_float2(key_f(key), __int_as_float(c * 8 + j));
      } else if (key == lo) {
        const int p = atomicAdd(&sh.s_nt, 1);
        if (p < SR_CAP - amax) sh.cand[SR_CAP - 1 - p] = make_float2(key_f(key), __int_as_float(c * 8 + j));
      }
    }
  }
  for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) {
    const unsigned key = bf_key(l[i]);
    if (key == 0u) continue;
    if (key > lo) {
      const int p = atomicAdd(&sh.s_n, 1);
      if (p < amax) sh.cand[p] = make_float2(key_f(key), __int_as_float(i));
    } else if (key == lo) {
      const int p = atomicAdd(&sh.s_nt, 1);
      if (p < SR_CAP - amax) sh.cand[SR_CAP - 1 - p] = make_float2(key_f(key), __int_as_float(i));
    }
  }
  __syncthreads();
  na = min(sh.s_n, amax);
  nt = min(sh.s_nt, SR_CAP - amax);
  }
  const int n = min(na, SR_CAP) + nt;
  // the ties (slots [SR_CAP - nt, SR_CAP)) move down behind the [0, na) block: one contiguous list
  if (nt > 0 && na < SR_CAP - nt) {
    float2 t[SR_CAP / SR_THREADS];
#pragma unroll
    for (int u = 0; u < SR_CAP / SR_THREADS; ++u) {
      const int j = tid + u * SR_THREADS;
      if (j < nt) t[u] = sh.cand[SR_CAP - nt + j];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < SR_CAP / SR_THREADS; ++u) {
      const int j = tid + u * SR_THREADS;
      if (j < nt) sh.cand[na + j] = t[u];
    }
    __syncthreads();
  }

  // ---- 3. rank = #strictly better candidates; ranks < k are the top-k.  Candidates are read 16 B
  // (two) at a time, 8 reads in flight (a dependent LDS round trip per candidate was ~8 us at
  // n ~ 150 and most of the k = 256 launch).
  const float4* c4 = reinterpret_cast<const float4*>(sh.cand);
  const int n2 = (n + 1) >> 1;
  for (int j = tid; j < n; j += SR_THREADS) {
    const float2 cj = sh.cand[j];
    const int ij = __float_as_int(cj.y);
    int r = 0;
    for (int i0 = 0; i0 < n2; i0 += 8) {
      float4 q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] = c4[min(i0 + u, n2 - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = 2 * (i0 + u);
        if (i0 + u < n2) {
          r += (q[u].x > cj.x || (q[u].x == cj.x && __float_as_int(q[u].y) < ij)) ? 1 : 0;
          if (i + 1 < n) r += (q[u].z > cj.x || (q[u].z == cj.x && __float_as_int(q[u].w) < ij)) ? 1 : 0;
        }
      }
    }
    if (r < k) { sh.i_r[r] = ij; sh.w_r[r] = cj.x; }
    if (r == 0) sh.s_m = cj.x;
  }
  __syncthreads();
  return n;
}

// Phase 4 (wave 0 only): softmax weights of ranks [0, kk) at temperature t, nucleus = shortest
// prefix with mass >= top_p, inverse-CDF pick with u = hash(seed, row).  Returns the picked rank
// (uniform in the wave), -1 when kk == 0.
static __device__ __forceinline__ int draw_rank(const SrShared& sh, int kk, float t, float top_p, unsigned seed,
                                                unsigned row) {
  const int lane = threadIdx.x & 63;
  if (kk <= 0) return -1;
  const float m = sh.s_m, it = 1.f / fmaxf(t, 1e-5f);
  float c4[4];
  float run = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 4 * lane + q;
    run += r < kk ? __expf((sh.w_r[r] - m) * it) : 0.f;
    c4[q] = run;                                  // lane-local inclusive prefix
  }
  float pre = run;                                // wave exclusive scan of lane totals
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(pre, o, 64);
    if (lane >= o) pre += y;
  }
  pre -= run;
  const float s = __shfl(pre + run, 63, 64);      // total mass of the top-k
  const float tp = top_p * s;
  int cut = kk;                                   // nucleus size = first rank with cum >= top_p, + 1
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 4 * lane + q;
    if (r < kk && pre + c4[q] >= tp) cut = min(cut, r + 1);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cut = min(cut, __shfl_xor(cut, o, 64));
  const int last = cut - 1;
  const float mass = __shfl(pre + c4[last & 3], last >> 2, 64);
  const float target = row_uniform(seed, row) * mass;
  int pick = last;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 4 * lane + q;
    if (r < cut && pre + c4[q] > target) pick = min(pick, r);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pick = min(pick, __shfl_xor(pick, o, 64));
  return pick;
}

__global__ void __launch_bounds__(SR_THREADS) sample_rows_kernel(const u16* __restrict__ logits, long stride, int V,
                                                                 const float* __restrict__ temp,
                                                                 const float* __restrict__ top_p,
                                                                 const int* __restrict__ top_k,
                                                                 const unsigned* __restrict__ seed,
                                                                 int* __restrict__ out) {
  __shared__ SrShared sh;
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const u16* l = logits + (long)row * stride;
  const int nv = V >> 3;
  const float t = temp[row];

  if (!(t > 0.f)) {  // greedy row: arg-max, ties -> lowest index
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    for_each_vec<SR_THREADS>(l, nv, tid, [&](const uint4 v, int c) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) better(bv, bi, f[j], c * 8 + j);
    });
    for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) better(bv, bi, bf2f(l[i]), i);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      better(bv, bi, ov, oi);
    }
    if (lane == 0) { sh.sv[wid] = bv; sh.si[wid] = bi; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < SR_THREADS / 64; ++w) better(bv, bi, sh.sv[w], sh.si[w]);
      out[row] = (bi == 0x7fffffff) ? 0 : bi;
    }
    return;
  }
  int k = top_k[row];
  if (k <= 0 || k > SR_KMAX) k = SR_KMAX;
  if (k > V) k = V;
  const int n = row_topk(l, V, k, sh);
  if (wid == 0) {
    const int pick = draw_rank(sh, min(k, n), t, top_p[row], *seed, (unsigned)row);
    if (lane == 0) out[row] = pick >= 0 ? sh.i_r[pick] : 0;   // an all-NaN row yields token 0
  }
}

// ---------------------------------------------------------------------------- vocab-parallel sampler
// Tensor parallelism shards the LM head by vocabulary: rank p holds logits [S, V/tp] of ids
// [start_p, start_p + V/tp).  The global top-k (k <= 256) of a row lies inside the union of every
// shard's top-256, so each rank reduces its shard to TP_KC ranked candidates (tp_cands_kernel), one
// all-gather moves [tp, S, TP_KC] (value, id) pairs, and tp_sample_kernel merges the tp sorted lists
// (rank of a candidate = its position in its list + a binary search in every other list, same
// (value desc, id asc) order as sample_rows_kernel) and runs the same draw — every rank holds the
// same gathered lists and the same seed, so every rank emits the same token, and it is the token
// sample_rows_kernel would draw from the unsharded row.
constexpr int TP_KC = 256;

// cand [S, TP_KC] int2 (value f32 bits, global id); ranks past the shard's candidate count are
// (-inf, INT_MAX)
__global__ void __launch_bounds__(SR_THREADS) tp_cands_kernel(const u16* __restrict__ logits, long stride, int V,
                                                              int start, int2* __restrict__ cand) {
  __shared__ SrShared sh;
  const int row = blockIdx.x, tid = threadIdx.x;
  const int k = min(TP_KC, V);
  const int n = min(row_topk(logits + (long)row * stride, V, k, sh), k);
  for (int r = tid; r < TP_KC; r += SR_THREADS)
    cand[(long)row * TP_KC + r] = r < n ? make_int2(__float_as_int(sh.w_r[r]), sh.i_r[r] + start)
                                        : make_int2(__float_as_int(-INFINITY), 0x7fffffff);
}

static __device__ __forceinline__ bool cand_better(int2 a, int2 b) {  // value desc, id asc
  const float va = __int_as_float(a.x), vb = __int_as_float(b.x);
  return va > vb || (va == vb && a.y < b.y);
}

// cands [tp][S][TP_KC] (rank-sorted lists of every shard, all-gathered); out [S] global token ids
__global__ void __launch_bounds__(SR_THREADS) tp_sample_kernel(const int2* __restrict__ cands, int S, int tp,
                                                               const float* __restrict__ temp,
                                                               const float* __restrict__ top_p,
                                                               const int* __restrict__ top_k,
                                                               const unsigned* __restrict__ seed,
                                                               int* __restrict__ out) {
  __shared__ SrShared sh;
  __shared__ int2 lists[8 * TP_KC];
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = tp * TP_KC;
  for (int j = tid; j < n; j += SR_THREADS) lists[j] = cands[((long)(j / TP_KC) * S + row) * TP_KC + j % TP_KC];
  __syncthreads();
  const float t = temp[row];
  int k = t > 0.f ? top_k[row] : 1;
  if (k <= 0 || k > SR_KMAX) k = SR_KMAX;
  if (tid == 0) sh.s_n = 0;
  __syncthreads();
  int valid = 0;
  for (int j = tid; j < n; j += SR_THREADS) {
    const int p = j / TP_KC, i = j % TP_KC;
    const int2 c = lists[j];
    if (c.y == 0x7fffffff) continue;                 // padding
    ++valid;
    int r = i;                                       // better ones in its own (sorted) list
    for (int q = 0; q < tp; ++q) {
      if (q == p) continue;
      int lo = 0, hi = TP_KC;                        // # of list q strictly better than c
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cand_better(lists[q * TP_KC + mid], c)) lo = mid + 1; else hi = mid;
      }
      r += lo;
    }
    if (r < k) { sh.i_r[r] = c.y; sh.w_r[r] = __int_as_float(c.x); }
    if (r == 0) sh.s_m = __int_as_float(c.x);
  }
  atomicAdd(&sh.s_n, valid);
  __syncthreads();
  const int kk = min(k, sh.s_n);
  if (wid == 0) {
    const int pick = t > 0.f ? draw_rank(sh, kk, t, top_p[row], *seed, (unsigned)row) : (kk > 0 ? 0 : -1);
    if (lane == 0) out[row] = pick >= 0 ? sh.i_r[pick] : 0;
  }
}
// ---------------------------------------------------------------------------- split-vocab sampler
// Small batches: one workgroup per row leaves ~250 CUs idle and puts a whole 32K-128K logit row
// behind one CU's load queue (batch-1 sampler: 10 us TinyLlama, 28 us Llama-3-8B,
// profiles/r3_single_stream_decode.md).  sample_split_kernel runs grid (P, B): workgroup (p, row)
// reduces vocab shard p of the row to its ranked top-k (k = the row's top_k; a greedy row: its
// arg-max), stores the list write-through and takes the row's ticket (recipe R1, common.h); the
// last arriver merges the P ranked lists (rank = position in its own list + a binary search in
// every other list, the tp_sample_kernel rule) and draws exactly as sample_rows_kernel does.  The
// global top-k lies inside the union of the shards' top-k, so the token is the one
// sample_rows_kernel picks from the whole row.
constexpr int SS_MAXP = 8;

// part: [B][P][SR_KMAX] int2 (value f32 bits, id) -- part_bytes covers it; counters [B], zero
// (re-armed by every last arriver)
__global__ void __launch_bounds__(SR_THREADS) sample_split_kernel(const u16* __restrict__ logits, long stride, int V,
                                                                  int P, int vs, const float* __restrict__ temp,
                                                                  const float* __restrict__ top_p,
                                                                  const int* __restrict__ top_k,
                                                                  const unsigned* __restrict__ seed, void* part,
                                                                  unsigned part_bytes, int* __restrict__ counters,
                                                                  int* __restrict__ out) {
  __shared__ SrShared sh;
  __shared__ int2 lists[SS_MAXP * SR_KMAX];
  __shared__ int s_last;
  const int p = blockIdx.x, row = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int start = p * vs, len = min(vs, V - start);
  const u16* l = logits + (long)row * stride + start;
  const float t = temp[row];
  const bool greedy = !(t > 0.f);
  int k = greedy ? 1 : top_k[row];
  if (k <= 0 || k > SR_KMAX) k = SR_KMAX;
  if (k > V) k = V;
  const int kp = (k + 1) & ~1;                    // list length: whole 16-B pairs
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(part, part_bytes);
  const unsigned base = (unsigned)(((long)row * P + p) * SR_KMAX * 8);
  if (greedy) {                                   // shard arg-max, ties -> lowest index
    float bv = -INFINITY;
    int bi = 0x7fffffff;
    const int nv = len >> 3;
    for_each_vec<SR_THREADS>(l, nv, tid, [&](const uint4 v, int c) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) better(bv, bi, f[j], start + c * 8 + j);
    });
    for (int i = (nv << 3) + tid; i < len; i += SR_THREADS) better(bv, bi, bf2f(l[i]), start + i);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      better(bv, bi, ov, oi);
    }
    if (lane == 0) { sh.sv[wid] = bv; sh.si[wid] = bi; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < SR_THREADS / 64; ++w) better(bv, bi, sh.sv[w], sh.si[w]);
      st_wt16(rs, base, make_float4(bv, __int_as_float(bi), -INFINITY, __int_as_float(0x7fffffff)));
    }
  } else {
    const int n = min(row_topk(l, len, min(k, len), sh), k);
    for (int r2 = tid; 2 * r2 < kp; r2 += SR_THREADS) {
      const int r = 2 * r2;
      const float v0 = r < n ? sh.w_r[r] : -INFINITY, v1 = r + 1 < n ? sh.w_r[r + 1] : -INFINITY;
      const int i0 = r < n ? sh.i_r[r] + start : 0x7fffffff, i1 = r + 1 < n ? sh.i_r[r + 1] + start : 0x7fffffff;
      st_wt16(rs, base + r * 8, make_float4(v0, __int_as_float(i0), v1, __int_as_float(i1)));
    }
  }
  if (!ticket_last(counters + row, P, &s_last)) return;

  // ---- last arriver of the row: gather the P lists, merge, draw
  const unsigned rbase = (unsigned)((long)row * P * SR_KMAX * 8);
  for (int j = tid; 2 * j < P * kp; j += SR_THREADS) {
    const int q = (2 * j) / kp, r = (2 * j) % kp;
    const float4 v = ld_wt16(rs, rbase + (unsigned)((q * SR_KMAX + r) * 8));
    lists[q * kp + r] = make_int2(__float_as_int(v.x), __float_as_int(v.y));
    lists[q * kp + r + 1] = make_int2(__float_as_int(v.z), __float_as_int(v.w));
  }
  if (tid == 0) sh.s_n = 0;
  __syncthreads();
  if (greedy) {
    if (tid == 0) {
      float bv = -INFINITY;
      int bi = 0x7fffffff;
      for (int q = 0; q < P; ++q) better(bv, bi, __int_as_float(lists[q * kp].x), lists[q * kp].y);
      out[row] = (bi == 0x7fffffff) ? 0 : bi;
    }
    return;
  }
  int valid = 0;
  for (int j = tid; j < P * kp; j += SR_THREADS) {
    const int q = j / kp, i = j % kp;
    const int2 c = lists[j];
    if (c.y == 0x7fffffff) continue;                 // padding
    ++valid;
    int r = i;                                       // better ones in its own (sorted) list
    for (int o = 0; o < P; ++o) {
      if (o == q) continue;
      int lo = 0, hi = kp;                           // # of list o strictly better than c
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cand_better(lists[o * kp + mid], c)) lo = mid + 1; else hi = mid;
      }
      r += lo;
    }
    if (r < k) { sh.i_r[r] = c.y; sh.w_r[r] = __int_as_float(c.x); }
    if (r == 0) sh.s_m = __int_as_float(c.x);
  }
  atomicAdd(&sh.s_n, valid);
  __syncthreads();
  const int kk = min(k, sh.s_n);
  if (wid == 0) {
    const int pick = draw_rank(sh, kk, t, top_p[row], *seed, (unsigned)row);
    if (lane == 0) out[row] = pick >= 0 ? sh.i_r[pick] : 0;
  }
}
}  // namespace

extern "C" int dllm_sample_split_maxp() { return SS_MAXP; }
extern "C" int dllm_sample_split_kmax() { return SR_KMAX; }

// logits [B, V] bf16 (row stride % 8 == 0) -> out [B]; P vocab shards of vs (% 8 == 0) logits each;
// part >= B * P * SR_KMAX int2, counters >= B ints, zero.  Same tokens as dllm_sample_rows.
extern "C" int dllm_sample_split(const void* logits, long stride, int B, int V, int P, const float* temp,
                                 const float* top_p, const int* top_k, const unsigned* seed, void* part,
                                 long part_bytes, int* counters, int* out, hipStream_t stream) {
  if (B <= 0) return 0;
  if (V <= 0 || stride % 8 != 0 || P < 1 || P > SS_MAXP) return -1;
  const int vs = ((V + P - 1) / P + 7) / 8 * 8;
  if ((long)(P - 1) * vs >= V) return -2;              // an empty shard: use fewer
  const long need = (long)B * P * SR_KMAX * 8;
  if (part_bytes < need || need > 0x7fffffffL) return -3;
  hipLaunchKernelGGL(sample_split_kernel, dim3(P, B), dim3(SR_THREADS), 0, stream, (const u16*)logits, stride, V, P,
                     vs, temp, top_p, top_k, seed, part, (unsigned)need, counters, out);
  return (int)hipGetLastError();
}

extern "C" int dllm_sample_rows(const void* logits, long stride, int B, int V, const float* temp, const float* top_p,
                                const int* top_k, const unsigned* seed, int* out, hipStream_t stream) {
  if (B <= 0) return 0;
  if (V <= 0 || stride % 8 != 0) return -1;
  hipLaunchKernelGGL(sample_rows_kernel, dim3(B), dim3(SR_THREADS), 0, stream, (const u16*)logits, stride, V, temp,
                     top_p, top_k, seed, out);
  return (int)hipGetLastError();
}

extern "C" int dllm_tp_cands_k() { return TP_KC; }

// logits [S, V] bf16 (row stride % 8 == 0) of a vocab shard starting at global id `start` -> cand [S, TP_KC] int2
extern "C" int dllm_tp_cands(const void* logits, long stride, int S, int V, int start, void* cand, hipStream_t stream) {
  if (S <= 0) return 0;
  if (V <= 0 || stride % 8 != 0) return -1;
  hipLaunchKernelGGL(tp_cands_kernel, dim3(S), dim3(SR_THREADS), 0, stream, (const u16*)logits, stride, V, start,
                     (int2*)cand);
  return (int)hipGetLastError();
}

// cands [tp, S, TP_KC] int2 -> out [S] token ids
extern "C" int dllm_tp_sample(const void* cands, int S, int tp, const float* temp, const float* top_p, const int* top_k,
                              const unsigned* seed, int* out, hipStream_t stream) {
  if (S <= 0) return 0;
  if (tp < 1 || tp > 8) return -1;
  hipLaunchKernelGGL(tp_sample_kernel, dim3(S), dim3(SR_THREADS), 0, stream, (const int2*)cands, S, tp, temp, top_p,
                     top_k, seed, out);
  return (int)hipGetLastError();
}

extern "C" int dllm_argmax(const void* logits, long stride, int B, int V, int is_bf16, int* out, hipStream_t stream) {
  if (B <= 0) return 0;
  if (is_bf16)
    hipLaunchKernelGGL(argmax_kernel<true>, dim3(B), dim3(256), 0, stream, logits, stride, V, out);
  else
    hipLaunchKernelGGL(argmax_kernel<false>, dim3(B), dim3(256), 0, stream, logits, stride, V, out);
  return (int)hipGetLastError();
}

extern "C" int dllm_sample_topp(const float* vals, const long* idx, int B, int K, const float* temp,
                                const float* top_p, const float* u, int* out, hipStream_t stream) {
  if (B <= 0) return 0;
  hipLaunchKernelGGL(sample_topp_kernel, dim3(B), dim3(64), 0, stream, vals, idx, K, temp, top_p, u, out);
  return (int)hipGetLastError();
}
