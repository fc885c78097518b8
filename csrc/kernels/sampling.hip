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

__global__ void __launch_bounds__(SR_THREADS) sample_rows_kernel(const u16* __restrict__ logits, long stride, int V,
                                                                 const float* __restrict__ temp,
                                                                 const float* __restrict__ top_p,
                                                                 const int* __restrict__ top_k,
                                                                 const unsigned* __restrict__ seed,
                                                                 int* __restrict__ out) {
  __shared__ unsigned hist[4096];
  __shared__ float2 cand[SR_CAP];          // (value, index bits)
  __shared__ float w_r[SR_KMAX];           // softmax weight by rank
  __shared__ int i_r[SR_KMAX];             // token id by rank
  __shared__ unsigned wsum[SR_THREADS / 64];
  __shared__ float sv[SR_THREADS / 64];
  __shared__ int si[SR_THREADS / 64];
  __shared__ int s_bin, s_above, s_n, s_nt, s_lo, s_amax;
  __shared__ float s_m;
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
    if (lane == 0) { sv[wid] = bv; si[wid] = bi; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < SR_THREADS / 64; ++w) better(bv, bi, sv[w], si[w]);
      out[row] = (bi == 0x7fffffff) ? 0 : bi;
    }
    return;
  }
  int k = top_k[row];
  if (k <= 0 || k > SR_KMAX) k = SR_KMAX;
  if (k > V) k = V;

  // ---- 0. fast bound (no histogram): T0 = the k-th largest of the 256 per-thread maximum keys.
  // At least k logits are >= T0 (one per thread whose maximum is), so every top-k logit is too;
  // when few logits reach T0 (typical: ~k-3k of 32 K) they are the whole candidate list and the
  // 4096-bin LDS-atomic histogram (hot bins serialise its atomics: ~40 us for one row) is skipped.
  // A flat row (> SR_MAXN logits at or above T0) falls through to the histogram path.
  {
    unsigned tmax = 0u;
    for_each_vec<SR_THREADS>(l, nv, tid, [&](const uint4 v, int) {
      const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) tmax = max(tmax, bf_key(e[j]));
    });
    for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) tmax = max(tmax, bf_key(l[i]));
    hist[tid] = tmax;
    if (tid == 0) s_n = 0;
    __syncthreads();
    int r = 0;  // rank among the thread maxima (ties -> lower thread first)
    for (int j = 0; j < SR_THREADS; ++j) {
      const unsigned o = hist[j];
      r += (o > tmax || (o == tmax && j < tid)) ? 1 : 0;
    }
    if (r == k - 1) s_lo = (int)tmax;
    __syncthreads();
    const unsigned t0 = (unsigned)s_lo;
    for_each_vec<SR_THREADS>(l, nv, tid, [&](const uint4 v, int c) {
      const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned key = bf_key(e[j]);
        if (key >= t0 && key != 0u) {
          const int p = atomicAdd(&s_n, 1);
          if (p < SR_CAP) cand[p] = make_float2(key_f(key), __int_as_float(c * 8 + j));
        }
      }
    });
    for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) {
      const unsigned key = bf_key(l[i]);
      if (key >= t0 && key != 0u) {
        const int p = atomicAdd(&s_n, 1);
        if (p < SR_CAP) cand[p] = make_float2(key_f(key), __int_as_float(i));
      }
    }
    __syncthreads();
  }
  int na, nt;
  if (s_n >= k && s_n <= SR_MAXN) {
    na = s_n;
    nt = 0;
  } else {
  __syncthreads();  // every thread has read s_n before the histogram path reuses it

  // ---- 1. coarse histogram (12-bit bins) and the bin of the k-th largest
  for (int i = tid; i < 4096; i += SR_THREADS) hist[i] = 0u;
  __syncthreads();
  for (int c = tid; c < nv; c += SR_THREADS) {
    const uint4 v = ld16(l + c * 8);
    const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) atomicAdd(&hist[bf_key(e[j]) >> 4], 1u);
  }
  for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) atomicAdd(&hist[bf_key(l[i]) >> 4], 1u);
  __syncthreads();
  unsigned mine = 0;  // thread t owns bins 4095-16t .. 4080-16t (descending key order)
#pragma unroll
  for (int j = 0; j < 16; ++j) mine += hist[4095 - 16 * tid - j];
  unsigned x = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  unsigned base = 0;
  for (int w = 0; w < wid; ++w) base += wsum[w];
  const unsigned incl = base + x, excl = incl - mine;
  if (excl < (unsigned)k && incl >= (unsigned)k) {  // exactly one thread
    unsigned acc = excl;
    for (int j = 0; j < 16; ++j) {
      const int b = 4095 - 16 * tid - j;
      if (acc + hist[b] >= (unsigned)k) { s_bin = b; s_above = (int)acc; break; }
      acc += hist[b];
    }
  }
  __syncthreads();
  const int bin = s_bin;
  if (s_above + (int)hist[bin] > SR_MAXN) {  // crowded bin: exact threshold from its low 4 bits
    __syncthreads();
    if (tid < 16) hist[tid] = 0u;            // hist[0..15] re-used as the 16 fine bins (the coarse
    __syncthreads();                         // counts are no longer needed past this point)
    for (int c = tid; c < nv; c += SR_THREADS) {
      const uint4 v = ld16(l + c * 8);
      const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned key = bf_key(e[j]);
        if ((int)(key >> 4) == bin) atomicAdd(&hist[key & 15], 1u);
      }
    }
    for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) {
      const unsigned key = bf_key(l[i]);
      if ((int)(key >> 4) == bin) atomicAdd(&hist[key & 15], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned acc = (unsigned)s_above;
      int lo = bin << 4;
      for (int b = 15; b >= 0; --b) {
        if (acc + hist[b] >= (unsigned)k) { lo = (bin << 4) | b; break; }
        acc += hist[b];
      }
      s_lo = lo;
      s_amax = (int)acc;  // exactly the keys strictly above lo (< k)
    }
  } else if (tid == 0) {
    s_lo = bin << 4;
    s_amax = s_above + (int)hist[bin];  // every candidate (<= SR_MAXN): none is ever dropped
  }
  if (tid == 0) { s_n = 0; s_nt = 0; }
  __syncthreads();

  // ---- 2. candidates: every logit at or above the threshold key.  Keys strictly above it (at most
  // s_amax: < k for a crowded bin, <= SR_MAXN otherwise) fill slots from the bottom; ties AT the
  // threshold fill slots from the top, never below slot s_amax — so a crowded tie bin can only
  // drop ties, never a strictly better logit, and the top-k stays exact.
  const unsigned lo = (unsigned)s_lo;
  const int amax = min(s_amax, SR_CAP);
  for (int c = tid; c < nv; c += SR_THREADS) {
    const uint4 v = ld16(l + c * 8);
    const u16* e = reinterpret_cast<const u16*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned key = bf_key(e[j]);
      if (key > lo) {
        const int p = atomicAdd(&s_n, 1);
        if (p < amax) cand[p] = make_float2(key_f(key), __int_as_float(c * 8 + j));
      } else if (key == lo) {
        const int p = atomicAdd(&s_nt, 1);
        if (p < SR_CAP - amax) cand[SR_CAP - 1 - p] = make_float2(key_f(key), __int_as_float(c * 8 + j));
      }
    }
  }
  for (int i = (nv << 3) + tid; i < V; i += SR_THREADS) {
    const unsigned key = bf_key(l[i]);
    if (key > lo) {
      const int p = atomicAdd(&s_n, 1);
      if (p < amax) cand[p] = make_float2(key_f(key), __int_as_float(i));
    } else if (key == lo) {
      const int p = atomicAdd(&s_nt, 1);
      if (p < SR_CAP - amax) cand[SR_CAP - 1 - p] = make_float2(key_f(key), __int_as_float(i));
    }
  }
  __syncthreads();
  na = min(s_n, amax);
  nt = min(s_nt, SR_CAP - amax);
  }
  const int n = na + nt;
  // candidate j of the union [0, na) u [SR_CAP - nt, SR_CAP)
  auto cidx = [&](int j) { return j < na ? j : SR_CAP - nt + (j - na); };

  // ---- 3. rank = #strictly better candidates; ranks < k are the top-k
  for (int j = tid; j < n; j += SR_THREADS) {
    const float2 cj = cand[cidx(j)];
    const int ij = __float_as_int(cj.y);
    int r = 0;
    for (int i = 0; i < n; ++i) {
      const float2 ci = cand[cidx(i)];
      r += (ci.x > cj.x || (ci.x == cj.x && __float_as_int(ci.y) < ij)) ? 1 : 0;
    }
    if (r < k) { i_r[r] = ij; w_r[r] = cj.x; }
    if (r == 0) s_m = cj.x;
  }
  __syncthreads();

  // ---- 4. temperature, nucleus, draw (wave 0; rank r = 4 * lane + q)
  if (wid == 0) {
    const int kk = min(k, n);
    const float m = s_m, it = 1.f / fmaxf(t, 1e-5f);
    float c4[4];
    float run = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 4 * lane + q;
      run += r < kk ? __expf((w_r[r] - m) * it) : 0.f;
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
    const float tp = top_p[row] * s;
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
    const float target = row_uniform(*seed, (unsigned)row) * mass;
    int pick = last;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 4 * lane + q;
      if (r < cut && pre + c4[q] > target) pick = min(pick, r);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pick = min(pick, __shfl_xor(pick, o, 64));
    if (lane == 0) out[row] = i_r[pick];
  }
}
}  // namespace

extern "C" int dllm_sample_rows(const void* logits, long stride, int B, int V, const float* temp, const float* top_p,
                                const int* top_k, const unsigned* seed, int* out, hipStream_t stream) {
  if (B <= 0) return 0;
  if (V <= 0 || stride % 8 != 0) return -1;
  hipLaunchKernelGGL(sample_rows_kernel, dim3(B), dim3(SR_THREADS), 0, stream, (const u16*)logits, stride, V, temp,
                     top_p, top_k, seed, out);
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
