// RMSNorm / LayerNorm with fused residual add (bf16 I/O, f32 math).
//
// One workgroup per row; each thread owns up to MAXV 16-byte vectors of the row in
// registers, so the row is read once and written once (plus the residual stream).
//   rmsnorm:   r = x (+ res);  res_out = r;  y = r * rsqrt(mean(r^2) + eps) * w
//   layernorm: r = x (+ res);  res_out = r;  y = (r - mean) * rsqrt(var + eps) * w + b
#include "common.h"

namespace {
constexpr int MAXV = 4;  // vectors (8 x bf16) per thread -> H <= 256 * 8 * 4 = 8192

template <bool LAYERNORM>
__global__ void __launch_bounds__(256) norm_kernel(const u16* __restrict__ x, const u16* __restrict__ res_in,
                                                   u16* __restrict__ res_out, const u16* __restrict__ w,
                                                   const u16* __restrict__ b, u16* __restrict__ y, int H,
                                                   long x_stride, long y_stride, float eps) {
  __shared__ float red[16];
  const long row = blockIdx.x;
  const int nvec = H >> 3;
  const u16* xr = x + row * x_stride;
  float v[MAXV][8];
  // weight (and bias) vectors are issued together with the row loads, so the epilogue after the
  // block reduction does not wait on a second dependent memory round trip
  uint4 wv[MAXV], bv[MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      wv[i] = ld16(w + c * 8);
      if (LAYERNORM) bv[i] = ld16(b + c * 8);
      unpack8(ld16(xr + c * 8), v[i]);
      if (res_in) {
        float r[8];
        unpack8(ld16(res_in + row * (long)H + c * 8), r);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] += r[j];
        // residual stream is kept in bf16: round, store, and normalise the rounded value
        uint4 pk = pack8(v[i]);
        st16(res_out + row * (long)H + c * 8, pk);
        unpack8(pk, v[i]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += LAYERNORM ? v[i][j] : v[i][j] * v[i][j];
    }
  }
  float mean = 0.f, rstd;
  if (LAYERNORM) {
    mean = block_sum(s, red) / H;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = threadIdx.x + i * blockDim.x;
      if (c < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) { float d = v[i][j] - mean; q += d * d; }
      }
    }
    rstd = rsqrtf(block_sum(q, red) / H + eps);
  } else {
    rstd = rsqrtf(block_sum(s, red) / H + eps);
  }
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      float wf[8], o[8];
      unpack8(wv[i], wf);
      if (LAYERNORM) {
        float bf[8];
        unpack8(bv[i], bf);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * wf[j] + bf[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rstd * wf[j];
      }
      st16(y + row * y_stride + c * 8, pack8(o));
    }
  }
}
}  // namespace

extern "C" int dllm_norm(const void* x, const void* res_in, void* res_out, const void* w, const void* b, void* y,
                         int rows, int H, long x_stride, long y_stride, float eps, int layernorm,
                         hipStream_t stream) {
  if (H % 8 != 0 || H > 256 * 8 * MAXV || rows <= 0) return -1;
  int threads = ((H / 8 + 63) / 64) * 64;
  if (threads > 256) threads = 256;
  if ((H / 8 + threads - 1) / threads > MAXV) return -2;
  if (layernorm)
    hipLaunchKernelGGL(norm_kernel<true>, dim3(rows), dim3(threads), 0, stream, (const u16*)x, (const u16*)res_in,
                       (u16*)res_out, (const u16*)w, (const u16*)b, (u16*)y, H, x_stride, y_stride, eps);
  else
    hipLaunchKernelGGL(norm_kernel<false>, dim3(rows), dim3(threads), 0, stream, (const u16*)x, (const u16*)res_in,
                       (u16*)res_out, (const u16*)w, (const u16*)b, (u16*)y, H, x_stride, y_stride, eps);
  return (int)hipGetLastError();
}
