// Token sampling on the logits of the last position of every sequence.
//   argmax_kernel      : greedy (temperature 0) — one workgroup per row, 16-B loads of bf16/f32
//                        logits, wave-shuffle arg-max (ties -> lowest index, like torch.argmax).
//   sample_topp_kernel : temperature + top-p (nucleus) sampling over the row's top-K candidates
//                        (values sorted descending, from a top-k pass), one wave per row,
//                        inverse-CDF draw with a per-row uniform u in [0,1).
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
}  // namespace

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
