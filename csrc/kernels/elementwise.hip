// Memory-bound elementwise / small-reduction kernels (all 16-B vectorised, f32 math):
//   silu_mul     : out[t, i] = silu(gu[t, i]) * gu[t, I + i]        (SwiGLU, fused gate|up GEMM output)
//   gelu         : y = 0.5 x (1 + erf(x / sqrt 2))                    (MiniLM FFN)
//   mean_pool_l2 : out[b] = normalize(sum_s mask[b,s] x[b,s,:] / sum_s mask[b,s])   (sentence embedding)
//   moe_gate_topk: softmax over E experts, top-k, renormalised weights (Mixtral routing)
//   embed        : out[t] = table[ids[t] - lo] if lo <= ids[t] < lo + rows else 0   (token embedding;
//                  the masked form is the vocab-parallel shard of a TP rank, summed by the all-reduce)
#include "common.h"

namespace {

__global__ void silu_mul_kernel(const u16* __restrict__ gu, u16* __restrict__ out, long T, int I, long in_stride) {
  // 32-bit index math (the launcher guarantees T * I / 8 < 2^30, so v + stride cannot overflow): a 64-bit divide is a long
  // software sequence on CDNA, a 32-bit one a handful of VALU ops
  const int nv = I >> 3;
  const int nvec = (int)(T * nv);
  for (int v = blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += gridDim.x * blockDim.x) {
    const int t = v / nv;
    const int c = (v - t * nv) * 8;
    float gf[8], uf[8], o[8];
    unpack8(ld16(gu + t * in_stride + c), gf);
    unpack8(ld16(gu + t * in_stride + I + c), uf);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = gf[j] / (1.f + __expf(-gf[j])) * uf[j];
    st16(out + t * (long)I + c, pack8(o));
  }
}

// one wave per token row, 16-B vectors; rows of a 288 GB-resident table are gathered straight to
// registers (a random-row gather reads at ~5.5 TB/s: MI355X_MICROARCH.md)
// ssq (optional): the row's sum of squares, ssq[t] — the first decoder layer's folded-RMSNorm row
// scale then needs no separate res_add_ssq pass over the embeddings (one launch less per step)
// sc_buf != nullptr: the LAST workgroup instead applies a decode step's block-table updates
// (scatter_pairs_kernel's job: dst[idx_i] = val_i for sc_buf = [n, idx0, val0, ...]), so a decode
// step starts with one launch instead of two (~4.5 us at batch 1, profiles/r3_single_stream_decode.md)
__global__ void __launch_bounds__(256) embed_kernel(const int* __restrict__ ids, const u16* __restrict__ table,
                                                    u16* __restrict__ out, long T, int H, long lo, long rows,
                                                    float* __restrict__ ssq, int* __restrict__ sc_dst,
                                                    const int* __restrict__ sc_buf, int sc_cap) {
  if (sc_buf != nullptr && blockIdx.x == gridDim.x - 1) {
    const int n = min(sc_buf[0], sc_cap);
    for (int i = threadIdx.x; i < n; i += blockDim.x) sc_dst[sc_buf[1 + 2 * i]] = sc_buf[2 + 2 * i];
    return;
  }
  const long t = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (t >= T) return;
  const long r = ids[t] - lo;
  const bool ok = r >= 0 && r < rows;
  const u16* src = table + (ok ? r : 0) * (long)H;
  u16* dst = out + t * (long)H;
  float s = 0.f;
  for (int c = (threadIdx.x & 63) * 8; c < H; c += 64 * 8) {
    const uint4 v = ok ? ld16(src + c) : make_uint4(0, 0, 0, 0);
    st16(dst + c, v);
    if (ssq) {
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s += f[j] * f[j];
    }
  }
  if (ssq) {
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) ssq[t] = s;
  }
}

__global__ void gelu_kernel(const u16* __restrict__ x, u16* __restrict__ y, long n8) {
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    float f[8];
    unpack8(ld16(x + v * 8), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = 0.5f * f[j] * (1.f + erff(f[j] * 0.70710678118654752f));
    st16(y + v * 8, pack8(f));
  }
}

__global__ void __launch_bounds__(256) mean_pool_l2_kernel(const u16* __restrict__ x, const int* __restrict__ lens,
                                                           float* __restrict__ out, int S, int H) {
  __shared__ float red[16];
  const int b = blockIdx.x;
  const int n = lens[b];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};  // H <= 4 * blockDim
  for (int s = 0; s < n; ++s) {
    const u16* row = x + ((long)b * S + s) * H;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = threadIdx.x + i * blockDim.x;
      if (h < H) acc[i] += bf2f(row[h]);
    }
  }
  float ss = 0.f;
  const float inv = n > 0 ? 1.f / n : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) { acc[i] *= inv; ss += acc[i] * acc[i]; }
  const float nrm = sqrtf(block_sum(ss, red));
  const float sc = 1.f / fmaxf(nrm, 1e-12f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int h = threadIdx.x + i * blockDim.x;
    if (h < H) out[(long)b * H + h] = acc[i] * sc;
  }
}

// one thread per token; E <= 64, k <= 8
__global__ void moe_gate_kernel(const float* __restrict__ logits, int T, int E, int k, int* __restrict__ ids,
                                float* __restrict__ w) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const float* l = logits + (long)t * E;
  unsigned long long used = 0ull;
  float sel[8];
  int sid[8];
  for (int i = 0; i < k; ++i) {
    float best = -INFINITY;
    int bi = 0;
    for (int e = 0; e < E; ++e)
      if (!((used >> e) & 1ull) && l[e] > best) { best = l[e]; bi = e; }
    used |= 1ull << bi;
    sel[i] = best;
    sid[i] = bi;
  }
  // softmax over all E then renormalise over the selected == softmax over the selected logits
  const float m = sel[0];
  float s = 0.f;
  for (int i = 0; i < k; ++i) { sel[i] = __expf(sel[i] - m); s += sel[i]; }
  for (int i = 0; i < k; ++i) { ids[(long)t * k + i] = sid[i]; w[(long)t * k + i] = sel[i] / s; }
}
// Fused router: logits[t, e] = x[t] . wg[e] in fp32 (one wave per token: each lane holds XC 8-wide
// chunks of its token's row in registers, every expert's dot product is summed in a fixed order and
// reduced with an xor butterfly), then the same top-k / renormalised softmax as moe_gate_kernel.
// A token's result depends only on its own row, never on how many tokens share the launch, so a
// padded graph batch routes exactly like an eager one (a vendor GEMM picks its reduction split by M).
template <int XC>
__global__ void __launch_bounds__(256) moe_router_kernel(const u16* __restrict__ x, long x_stride,
                                                         const u16* __restrict__ wg, int T, int E, int H, int k,
                                                         int* __restrict__ ids, float* __restrict__ w,
                                                         float* __restrict__ logits) {
  __shared__ float lg[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int t = blockIdx.x * 4 + wv;
  if (t >= T) return;  // whole wave; no block barrier below
  const int nc = H >> 3;
  float xf[XC][8];
#pragma unroll
  for (int c = 0; c < XC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) unpack8(ld16(x + (long)t * x_stride + 8 * ch), xf[c]);
    else for (int q = 0; q < 8; ++q) xf[c][q] = 0.f;
  }
  for (int e = 0; e < E; ++e) {
    uint4 wv8[XC];
#pragma unroll
    for (int c = 0; c < XC; ++c) {
      const int ch = lane + 64 * c;
      wv8[c] = ch < nc ? ld16(wg + (long)e * H + 8 * ch) : make_uint4(0u, 0u, 0u, 0u);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < XC; ++c) {
      float f[8];
      unpack8(wv8[c], f);
#pragma unroll
      for (int q = 0; q < 8; ++q) s += xf[c][q] * f[q];
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
    if (lane == 0) lg[wv][e] = s;
  }
  if (lane != 0) return;
  const float* l = lg[wv];
  if (logits != nullptr)
    for (int e = 0; e < E; ++e) logits[(long)t * E + e] = l[e];
  unsigned long long used = 0ull;
  float sel[8];
  int sid[8];
  for (int i = 0; i < k; ++i) {
    float best = -INFINITY;
    int bi = 0;
    for (int e = 0; e < E; ++e)
      if (!((used >> e) & 1ull) && l[e] > best) { best = l[e]; bi = e; }
    used |= 1ull << bi;
    sel[i] = best;
    sid[i] = bi;
  }
  const float m = sel[0];
  float s = 0.f;
  for (int i = 0; i < k; ++i) { sel[i] = __expf(sel[i] - m); s += sel[i]; }
  for (int i = 0; i < k; ++i) { ids[(long)t * k + i] = sid[i]; w[(long)t * k + i] = sel[i] / s; }
}

// buf = [n, idx0, val0, idx1, val1, ...]: dst[idx_i] = val_i.  n is read on the device, so a
// captured decode graph applies a different number of block-table updates on every replay.
__global__ void scatter_pairs_kernel(int* __restrict__ dst, const int* __restrict__ buf, int cap) {
  const int n = min(buf[0], cap);
  for (int i = threadIdx.x; i < n; i += blockDim.x) dst[buf[1 + 2 * i]] = buf[2 + 2 * i];
}
}  // namespace

// ---- decode-step I/O inside the step's graph (round 4).  The step's inputs are staged by the host
// in pinned, device-mapped memory and its sampled tokens are read back from pinned memory; moving
// them with these kernels instead of hipMemcpyAsync keeps every decode step ONE graph launch on
// one queue: an async H2D copy runs on an SDMA engine and waited ~320 us per step for the
// read-back blit of the previous step to signal it (profiles/r4_driver_window_gaps.md).
// step_fetch: dec_dev[0:n_dec] <- dec_host, except the input ids, which the pipelined decode takes
// from the previous step's sampled tokens still on the device: ids[i] = d_out[src[i]] where
// src[i] >= 0 (src lives in the host buffer at src_off); and the attention work list
// items_dev <- items_host, as many words as its header says (decode_work_items layout).
__global__ void __launch_bounds__(256) step_fetch_kernel(const int* __restrict__ dec_host, int* __restrict__ dec_dev,
                                                         int n_dec, int ids_off, int src_off, int n_ids,
                                                         const int* __restrict__ d_out,
                                                         const int* __restrict__ items_host,
                                                         int* __restrict__ items_dev, int items_cap) {
  const int stride = gridDim.x * blockDim.x;
  const int gid = blockIdx.x * blockDim.x + threadIdx.x;
  int n_items = 0;
  if (items_host != nullptr) {
    const int h = items_host[0];
    n_items = min(h < 0 ? 4 + 4 * (-h) : 1 + 2 * h, items_cap);
  }
  for (int w = gid; w < n_dec; w += stride) {
    int v = dec_host[w];
    const int i = w - ids_off;
    if (i >= 0 && i < n_ids) {
      const int s = dec_host[src_off + i];
      if (s >= 0 && s < n_ids) v = d_out[s];
    }
    dec_dev[w] = v;
  }
  for (int w = gid; w < n_items; w += stride) items_dev[w] = items_host[w];
}

// step_store: out_host[0:n] <- d_out (the sampled tokens, + the TP health vote), last node of the graph
__global__ void __launch_bounds__(256) step_store_kernel(const int* __restrict__ d_out, int* __restrict__ out_host,
                                                         int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out_host[i] = d_out[i];
}

static inline int grid_for(long n, int threads) {
  long g = (n + threads - 1) / threads;
  if (g > 65536) g = 65536;
  return g < 1 ? 1 : (int)g;
}

extern "C" int dllm_silu_mul(const void* gu, void* out, long T, int I, long in_stride, hipStream_t stream) {
  if (I % 8 != 0) return -1;
  const long n = T * (I / 8);
  if (n == 0) return 0;
  if (n >= (1L << 30)) return -2;
  hipLaunchKernelGGL(silu_mul_kernel, dim3(grid_for(n, 256)), dim3(256), 0, stream, (const u16*)gu, (u16*)out, T, I,
                     in_stride);
  return (int)hipGetLastError();
}

extern "C" int dllm_embed(const int* ids, const void* table, void* out, long T, int H, long lo, long rows,
                          float* ssq, int* sc_dst, const int* sc_buf, int sc_cap, hipStream_t stream) {
  if (H % 8 != 0) return -1;
  if (T == 0 && sc_buf == nullptr) return 0;
  const unsigned grid = (unsigned)((T + 3) / 4) + (sc_buf != nullptr ? 1u : 0u);
  hipLaunchKernelGGL(embed_kernel, dim3(grid), dim3(256), 0, stream, ids, (const u16*)table, (u16*)out, T, H, lo, rows,
                     ssq, sc_dst, sc_buf, sc_cap);
  return (int)hipGetLastError();
}

extern "C" int dllm_gelu(const void* x, void* y, long n, hipStream_t stream) {
  if (n % 8 != 0) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(gelu_kernel, dim3(grid_for(n / 8, 256)), dim3(256), 0, stream, (const u16*)x, (u16*)y, n / 8);
  return (int)hipGetLastError();
}

extern "C" int dllm_mean_pool_l2(const void* x, const int* lens, float* out, int B, int S, int H, hipStream_t stream) {
  int threads = ((H + 3) / 4 + 63) / 64 * 64;
  if (threads > 256 || threads * 4 < H) return -1;
  hipLaunchKernelGGL(mean_pool_l2_kernel, dim3(B), dim3(threads), 0, stream, (const u16*)x, lens, out, S, H);
  return (int)hipGetLastError();
}

extern "C" int dllm_scatter_pairs(int* dst, const int* buf, int cap, hipStream_t stream) {
  hipLaunchKernelGGL(scatter_pairs_kernel, dim3(1), dim3(256), 0, stream, dst, buf, cap);
  return (int)hipGetLastError();
}

extern "C" int dllm_moe_gate(const float* logits, int T, int E, int k, int* ids, float* w, hipStream_t stream) {
  if (E > 64 || k > 8 || k > E) return -1;
  if (T == 0) return 0;
  hipLaunchKernelGGL(moe_gate_kernel, dim3((T + 127) / 128), dim3(128), 0, stream, logits, T, E, k, ids, w);
  return (int)hipGetLastError();
}

extern "C" int dllm_moe_router(const void* x, long x_stride, const void* wg, int T, int E, int H, int k, int* ids,
                               float* w, float* logits, hipStream_t stream) {
  if (E > 64 || k > 8 || k > E || H % 8 != 0 || H > 8192 || x_stride % 8 != 0) return -1;
  if (T == 0) return 0;
  const dim3 grid((T + 3) / 4), block(256);
  const int nc = H / 8;
  if (nc <= 256)
    hipLaunchKernelGGL(moe_router_kernel<4>, grid, block, 0, stream, (const u16*)x, x_stride, (const u16*)wg, T, E, H,
                       k, ids, w, logits);
  else if (nc <= 512)
    hipLaunchKernelGGL(moe_router_kernel<8>, grid, block, 0, stream, (const u16*)x, x_stride, (const u16*)wg, T, E, H,
                       k, ids, w, logits);
  else
    hipLaunchKernelGGL(moe_router_kernel<16>, grid, block, 0, stream, (const u16*)x, x_stride, (const u16*)wg, T, E,
                       H, k, ids, w, logits);
  return (int)hipGetLastError();
}

extern "C" int dllm_step_fetch(const int* dec_host, int* dec_dev, int n_dec, int ids_off, int src_off, int n_ids,
                               const int* d_out, const int* items_host, int* items_dev, int items_cap,
                               hipStream_t stream) {
  if (n_dec <= 0 || ids_off < 0 || src_off < 0 || ids_off + n_ids > n_dec || src_off + n_ids > n_dec) return -1;
  if ((items_host == nullptr) != (items_dev == nullptr)) return -2;
  hipLaunchKernelGGL(step_fetch_kernel, dim3(32), dim3(256), 0, stream, dec_host, dec_dev, n_dec, ids_off, src_off,
                     n_ids, d_out, items_host, items_dev, items_cap);
  return (int)hipGetLastError();
}

extern "C" int dllm_step_store(const int* d_out, int* out_host, int n, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(step_store_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, d_out, out_host, n);
  return (int)hipGetLastError();
}
