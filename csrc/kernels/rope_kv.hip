// Fused RoPE (rotate-half convention) + paged KV-cache write.
//
// Input: the fused QKV projection output, row t = [q(nq*d) | k(nkv*d) | v(nkv*d)] (bf16).
// Output: rotated q -> q_out [T, nq, d]; rotated k -> K cache; v -> transposed V cache.
// Cache layouts (per layer, BS = tokens per block):
//   K : [num_blocks][nkv][BS][d]   (key rows contiguous: the QK^T MFMA A-operand is a 16-B load)
//   Vt: [num_blocks][nkv][d][BS]   (keys contiguous per dim: the PV MFMA operand is an 8-B load)
// cos_sin: [max_pos][d] f32, first d/2 = cos, second d/2 = sin (host-precomputed table,
// cdna_hip_programming.md App. B 'Element-wise': no on-device trig).
// slot_mapping[t] = block * BS + offset, or < 0 to skip the cache write (padding rows).
#include "common.h"

namespace {

__global__ void __launch_bounds__(256) rope_kv_kernel(const u16* __restrict__ qkv, long qkv_stride,
                                                      const int* __restrict__ pos, const float* __restrict__ cos_sin,
                                                      const int* __restrict__ slots, u16* __restrict__ q_out,
                                                      u16* __restrict__ kc, u16* __restrict__ vc, int nq, int nkv,
                                                      int d, int BS) {
  const int t = blockIdx.x;
  const int half = d >> 1;
  const int upairs = half >> 3;        // 8-wide units per half-head
  const int n_rope = (nq + nkv) * upairs;
  const int n_v = nkv * (d >> 3);
  const u16* row = qkv + (long)t * qkv_stride;
  const int p = pos[t];
  const int slot = slots[t];
  const long blk = slot >= 0 ? slot / BS : 0;
  const int off = slot >= 0 ? slot % BS : 0;
  const float* cs = cos_sin + (long)p * d;
  for (int u = threadIdx.x; u < n_rope + n_v; u += blockDim.x) {
    if (u < n_rope) {
      const int h = u / upairs, i0 = (u % upairs) * 8;  // h < nq: query head; else key head h-nq
      const u16* src = row + h * d;
      float x1[8], x2[8], c[8], s[8], o1[8], o2[8];
      unpack8(ld16(src + i0), x1);
      unpack8(ld16(src + half + i0), x2);
#pragma unroll
      for (int j = 0; j < 8; ++j) { c[j] = cs[i0 + j]; s[j] = cs[half + i0 + j]; }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o1[j] = x1[j] * c[j] - x2[j] * s[j];
        o2[j] = x2[j] * c[j] + x1[j] * s[j];
      }
      if (h < nq) {
        u16* dst = q_out + ((long)t * nq + h) * d;
        st16(dst + i0, pack8(o1));
        st16(dst + half + i0, pack8(o2));
      } else if (slot >= 0) {
        const int kh = h - nq;
        u16* dst = kc + ((blk * nkv + kh) * BS + off) * (long)d;
        st16(dst + i0, pack8(o1));
        st16(dst + half + i0, pack8(o2));
      }
    } else if (slot >= 0) {
      const int uv = u - n_rope;
      const int kh = uv / (d >> 3), i0 = (uv % (d >> 3)) * 8;
      uint4 v = ld16(row + (nq + nkv + kh) * d + i0);
      const u16* vs = reinterpret_cast<const u16*>(&v);
      u16* dst = vc + (blk * nkv + kh) * (long)d * BS + off;
#pragma unroll
      for (int j = 0; j < 8; ++j) dst[(long)(i0 + j) * BS] = vs[j];
    }
  }
}

// K/V-only cache write (no rope) for already-rotated keys, e.g. KV hand-off between pools.
__global__ void kv_write_kernel(const u16* __restrict__ k, const u16* __restrict__ v, long kv_stride,
                                const int* __restrict__ slots, u16* __restrict__ kc, u16* __restrict__ vc, int nkv,
                                int d, int BS) {
  const int t = blockIdx.x;
  const int slot = slots[t];
  if (slot < 0) return;
  const long blk = slot / BS;
  const int off = slot % BS;
  const int nu = nkv * (d >> 3);
  for (int u = threadIdx.x; u < nu; u += blockDim.x) {
    const int kh = u / (d >> 3), i0 = (u % (d >> 3)) * 8;
    st16(kc + ((blk * nkv + kh) * BS + off) * (long)d + i0, ld16(k + t * kv_stride + kh * d + i0));
    uint4 vv = ld16(v + t * kv_stride + kh * d + i0);
    const u16* vs = reinterpret_cast<const u16*>(&vv);
    u16* dst = vc + (blk * nkv + kh) * (long)d * BS + off;
#pragma unroll
    for (int j = 0; j < 8; ++j) dst[(long)(i0 + j) * BS] = vs[j];
  }
}
}  // namespace

extern "C" int dllm_rope_kv(const void* qkv, long qkv_stride, const int* pos, const float* cos_sin, const int* slots,
                            void* q_out, void* kc, void* vc, int T, int nq, int nkv, int d, int BS,
                            hipStream_t stream) {
  if (d % 16 != 0 || T <= 0) return -1;
  const int units = (nq + nkv) * (d / 16) + nkv * (d / 8);
  int threads = ((units + 63) / 64) * 64;
  if (threads > 256) threads = 256;
  hipLaunchKernelGGL(rope_kv_kernel, dim3(T), dim3(threads), 0, stream, (const u16*)qkv, qkv_stride, pos, cos_sin,
                     slots, (u16*)q_out, (u16*)kc, (u16*)vc, nq, nkv, d, BS);
  return (int)hipGetLastError();
}

extern "C" int dllm_kv_write(const void* k, const void* v, long kv_stride, const int* slots, void* kc, void* vc,
                             int T, int nkv, int d, int BS, hipStream_t stream) {
  if (d % 8 != 0 || T <= 0) return -1;
  hipLaunchKernelGGL(kv_write_kernel, dim3(T), dim3(64), 0, stream, (const u16*)k, (const u16*)v, kv_stride, slots,
                     (u16*)kc, (u16*)vc, nkv, d, BS);
  return (int)hipGetLastError();
}
