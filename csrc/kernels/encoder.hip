// Router sentence encoder (MiniLM / BERT) kernels: bidirectional attention over a padded batch
// and the fused embedding sum + LayerNorm.  The projections run on tgemm.hip (bias / GELU /
// residual epilogues); LayerNorm after each residual on norm.hip; pooling on cosine.hip.
//
// Reference parity: the reference encodes every query with sentence-transformers
// all-MiniLM-L6-v2 on the host (/root/reference/src/query_router_engine.py:181,571).
//
// encoder_attn: qkv [B*S, 3H] (row b*S + s; q | k | v, head h at columns h*D), lens [B] -> out [B*S, H].
//   Workgroup = (64-query slice, head, sequence), 4 waves x 16 queries.  The head's K and V^T for
//   the whole sequence are staged once in LDS (S <= 512: <= 68 KB) and shared by the 4 waves.
//   Per 32-key chunk a wave computes S^T = K . Q^T with mfma_f32_16x16x32_bf16 (keys as rows:
//   every lane then holds the scores of ONE query, so the online softmax is lane-local plus two
//   xor-shuffles) and O^T += V^T . P^T with P^T taken straight from the score registers (key
//   permutation k-slot 8g+j <-> key j < 4 ? 4g+j : 16+4g+j-4, the same trick as attention.hip).
//   Keys >= lens[b] are masked (padding tokens); K/V rows past S are zero in LDS.
#include "common.h"

namespace {
constexpr float LOG2E = 1.4426950408889634f;

template <int D>
__global__ void __launch_bounds__(256) encoder_attn_kernel(const u16* __restrict__ qkv, const int* __restrict__ lens,
                                                           u16* __restrict__ out, int S, int SP, int nh,
                                                           float scale_log2) {
  constexpr int KSTEPS = D / 32, NT = D / 16, CPR = D / 8;  // 16-B chunks per head row
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int VLD = SP + 8;  // V^T row stride (bf16): 16-B pad against bank conflicts
  u16* sk = reinterpret_cast<u16*>(smem);    // [SP][D]
  u16* sv = sk + SP * D;                     // [D][VLD]
  const int b = blockIdx.z, h = blockIdx.y;
  const int H = nh * D;
  const long ld = 3L * H;
  const u16* base = qkv + (long)b * S * ld;
  const int len = min(lens[b], S);

  // ---- stage K rows and V^T for the whole sequence (zero past S)
  for (int e = threadIdx.x; e < SP * CPR; e += blockDim.x) {
    const int key = e / CPR, c = (e % CPR) * 8;
    uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
    if (key < S) {
      kv = ld16(base + (long)key * ld + H + h * D + c);
      vv = ld16(base + (long)key * ld + 2 * H + h * D + c);
    }
    st16(sk + key * D + c, kv);
    const uint32_t w[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sv[(c + 2 * j) * VLD + key] = (u16)(w[j] & 0xffffu);
      sv[(c + 2 * j + 1) * VLD + key] = (u16)(w[j] >> 16);
    }
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, rl = lane & 15;
  const int q0 = (int)blockIdx.x * 64 + wave * 16;  // this wave's first query row
  const int q = q0 + rl;                             // this lane's query row
  if (q0 >= S) return;                               // wave-uniform: no barrier follows
  bf16x8 qf[KSTEPS];
#pragma unroll
  for (int s = 0; s < KSTEPS; ++s)
    qf[s] = __builtin_bit_cast(bf16x8, q < S ? ld16(base + (long)q * ld + h * D + 8 * g + 32 * s) : make_uint4(0, 0, 0, 0));

  f32x4 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;
  for (int kc = 0; kc < len; kc += 32) {
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      const bf16x8 k0 = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sk + (kc + rl) * D + 8 * g + 32 * s));
      const bf16x8 k1 =
          __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sk + (kc + 16 + rl) * D + 8 * g + 32 * s));
      s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k0, qf[s], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(k1, qf[s], s1, 0, 0, 0);
    }
    float p[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      p[e] = (kc + 4 * g + e < len) ? s0[e] * scale_log2 : -INFINITY;
      p[4 + e] = (kc + 16 + 4 * g + e < len) ? s1[e] * scale_log2 : -INFINITY;
    }
    float mloc = p[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) mloc = fmaxf(mloc, p[j]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);  // finite: key kc < len is always valid
    const float alpha = exp2f(m_run - m_new);
    float lsum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { p[j] = exp2f(p[j] - m_new); lsum += p[j]; }
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    l_run = l_run * alpha + lsum;
    m_run = m_new;
    const bf16x8 pf = __builtin_bit_cast(bf16x8, pack8(p));
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const u16* vr = sv + (16 * n + rl) * VLD + kc + 4 * g;
      const uint2 a0 = *reinterpret_cast<const uint2*>(vr), a1 = *reinterpret_cast<const uint2*>(vr + 16);
      const uint4 vv = make_uint4(a0.x, a0.y, a1.x, a1.y);
      acc[n] *= alpha;
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, acc[n], 0, 0, 0);
    }
  }
  if (q >= S) return;
  // acc[n][e] = O^T[dim 16n + 4g + e][query rl]: 4 consecutive dims -> one 8-B store
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  u16* op = out + ((long)b * S + q) * H + h * D;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const uint32_t lo = (uint32_t)f2bf(acc[n][0] * inv) | ((uint32_t)f2bf(acc[n][1] * inv) << 16);
    const uint32_t hi = (uint32_t)f2bf(acc[n][2] * inv) | ((uint32_t)f2bf(acc[n][3] * inv) << 16);
    *reinterpret_cast<uint2*>(op + 16 * n + 4 * g) = make_uint2(lo, hi);
  }
}

// out[t] = LayerNorm(word[ids[t]] + pos[t % S] + type0) * w + b   (one wave per token, H <= 2048)
__global__ void __launch_bounds__(256) embed_ln_kernel(const int* __restrict__ ids, const u16* __restrict__ word,
                                                       const u16* __restrict__ pos, const u16* __restrict__ type0,
                                                       const u16* __restrict__ w, const u16* __restrict__ bias,
                                                       u16* __restrict__ out, int T, int S, int H, int vocab, float eps) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (t >= T) return;
  const int id = min(max(ids[t], 0), vocab - 1);
  const u16* wr = word + (long)id * H;
  const u16* pr = pos + (long)(t % S) * H;
  float x[4][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c < H) {
      float a[8], p[8], y[8];
      unpack8(ld16(wr + c), a);
      unpack8(ld16(pr + c), p);
      unpack8(ld16(type0 + c), y);
#pragma unroll
      for (int j = 0; j < 8; ++j) { x[i][j] = a[j] + p[j] + y[j]; s += x[i][j]; }
    }
  }
  const float mean = wave_sum(s) / H;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if ((lane + 64 * i) * 8 < H)
#pragma unroll
      for (int j = 0; j < 8; ++j) { const float d = x[i][j] - mean; v += d * d; }
  const float rstd = rsqrtf(wave_sum(v) / H + eps);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = (lane + 64 * i) * 8;
    if (c < H) {
      float gw[8], gb[8], y[8];
      unpack8(ld16(w + c), gw);
      unpack8(ld16(bias + c), gb);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = (x[i][j] - mean) * rstd * gw[j] + gb[j];
      st16(out + (long)t * H + c, pack8(y));
    }
  }
}
}  // namespace

extern "C" int dllm_encoder_attention(const void* qkv, const int* lens, void* out, int B, int S, int nh, int d,
                                      float scale, hipStream_t stream) {
  if (B <= 0 || S <= 0) return 0;
  if (S > 512) return -1;
  const int SP = (S + 31) / 32 * 32;
  const size_t lds = (size_t)SP * d * 2 + (size_t)d * (SP + 8) * 2;
  const dim3 grid((S + 63) / 64, nh, B);
  static const int attr_rc = [] {  // allow > 64 KB of dynamic LDS (S up to 512)
    int rc = (int)hipFuncSetAttribute((const void*)encoder_attn_kernel<32>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    rc |= (int)hipFuncSetAttribute((const void*)encoder_attn_kernel<64>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return rc;
  }();
  if (attr_rc != 0 && lds > 64 * 1024) return -3;
  switch (d) {
    case 32:
      hipLaunchKernelGGL(encoder_attn_kernel<32>, grid, dim3(256), lds, stream, (const u16*)qkv, lens, (u16*)out, S, SP,
                         nh, scale * LOG2E);
      break;
    case 64:
      hipLaunchKernelGGL(encoder_attn_kernel<64>, grid, dim3(256), lds, stream, (const u16*)qkv, lens, (u16*)out, S, SP,
                         nh, scale * LOG2E);
      break;
    default:
      return -2;
  }
  return (int)hipGetLastError();
}

extern "C" int dllm_embed_ln(const int* ids, const void* word, const void* pos, const void* type0, const void* w,
                             const void* b, void* out, int T, int S, int H, int vocab, float eps, hipStream_t stream) {
  if (H % 8 || H > 2048) return -1;
  if (T <= 0) return 0;
  hipLaunchKernelGGL(embed_ln_kernel, dim3((T + 3) / 4), dim3(256), 0, stream, ids, (const u16*)word, (const u16*)pos,
                     (const u16*)type0, (const u16*)w, (const u16*)b, (u16*)out, T, S, H, vocab, eps);
  return (int)hipGetLastError();
}
