// Paged attention for prefill, prefix-cached (chunked) prefill and decode — one MFMA kernel.
//
// Work unit: a 16-row query tile of ONE kv head.  Rows pack (token, head-in-GQA-group):
// row r -> token tok0 + r / G, query head kvh * G + r % G, so every K/V tile read from HBM
// serves all G query heads of its group (decode: 1 token x G heads; prefill: 16/G tokens x G).
//
// Per 32-key chunk (= two 16-token KV blocks) a wave computes
//   S^T[32 keys][16 rows] = K . Q^T         2 x (d/32) mfma_f32_16x16x32_bf16
//   online softmax per row (row = lane & 15, lane-local state, 2 xor-shuffles per reduction)
//   O^T[d][16 rows]      += V^T . P^T      (d/16) mfma_f32_16x16x32_bf16
// With S computed transposed, each lane already holds P for ITS row in the B-operand order of
// the PV product (the accumulator-as-operand trick, cdna_hip_programming.md §3), after the
// key permutation  k-slot 8g+j  <->  key (j<4 ? 4g+j : 16+4g+j-4).  The V cache is stored
// transposed per block ([d][16]), so the V^T operand is two 8-byte loads per lane and the K
// operand one 16-byte load per lane: no LDS staging, no transposes (decode is a memory-bound
// GEMV-like stream: App. B 'Attention decode', K/V straight to VGPRs).
//
// Split-K: grid.z splits the key range of every tile; 4 waves of a workgroup interleave 32-key
// chunks of the split and are combined through LDS.  With grid.z == 1 the workgroup writes the
// normalised bf16 output; otherwise it writes (m, l, O) partials and attn_combine_kernel reduces.
#include "common.h"

namespace {
constexpr int BS = 16;     // tokens per KV block
constexpr int WAVES = 4;
constexpr float LOG2E = 1.4426950408889634f;

struct AttnArgs {
  const u16* q;          // [Tq, nq, d]
  const u16* kc;         // [blocks, nkv, 16, d]
  const u16* vc;         // [blocks, nkv, d, 16]
  const int* block_tables;  // [num_seqs, max_blocks]
  const int* seq_qstart;
  const int* seq_qlen;
  const int* seq_ctx;
  const int* tile_seq;   // [num_tiles]  (< 0: padding tile)
  const int* tile_tok0;  // [num_tiles]
  u16* out;              // [Tq, nq, d]
  float* part_o;         // [num_tiles, nkv, splits, 16, d]
  float* part_ml;        // [num_tiles, nkv, splits, 16, 2]
  int nq, nkv, G, max_blocks, causal;
  float scale_log2;
};

template <int D>
__global__ void __launch_bounds__(256) paged_attn_kernel(AttnArgs a) {
  constexpr int KSTEPS = D / 32;
  constexpr int NT = D / 16;
  __shared__ float s_o[WAVES][16][D + 1];
  __shared__ float s_m[WAVES][16];
  __shared__ float s_l[WAVES][16];

  const int tile = blockIdx.x, kvh = blockIdx.y, split = blockIdx.z, splits = gridDim.z;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, rl = lane & 15;
  const int seq = a.tile_seq[tile];
  const int G = a.G, tpt = 16 / G;
  const int tok0 = a.tile_tok0[tile];
  int qlen = 0, ctx = 0, qstart = 0;
  if (seq >= 0) { qlen = a.seq_qlen[seq]; ctx = a.seq_ctx[seq]; qstart = a.seq_qstart[seq]; }

  // this lane's row
  const int my_tok = tok0 + rl / G, my_head = kvh * G + rl % G;
  const bool row_ok = seq >= 0 && my_tok < qlen;
  const int row_lim = !row_ok ? 0 : (a.causal ? ctx - qlen + my_tok + 1 : ctx);
  int last_tok = min(tok0 + tpt, qlen) - 1;
  int kmax = (seq < 0 || last_tok < tok0) ? 0 : (a.causal ? ctx - qlen + last_tok + 1 : ctx);
  int chunk = (kmax + splits - 1) / splits;
  chunk = (chunk + 31) & ~31;
  const int k_begin = split * chunk;
  const int k_end = min(kmax, k_begin + chunk);

  // Q fragments (B operand of S^T = K Q^T): row rl, dims 8g + j + 32*step
  bf16x8 qf[KSTEPS];
  {
    const u16* qp = a.q + ((long)(qstart + my_tok) * a.nq + my_head) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      uint4 v = row_ok ? ld16(qp + 32 * s) : make_uint4(0, 0, 0, 0);
      qf[s] = __builtin_bit_cast(bf16x8, v);
    }
  }

  f32x4 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  const int* bt = a.block_tables + (long)(seq >= 0 ? seq : 0) * a.max_blocks;
  const long head_stride = (long)BS * D;  // elements per (block, head) in either cache
  for (int kb = k_begin + 32 * wave; kb < k_end; kb += 32 * WAVES) {
    const int b0 = bt[kb >> 4];
    const int b1 = (kb + 16 < k_end) ? bt[(kb >> 4) + 1] : b0;
    const u16* k0 = a.kc + ((long)b0 * a.nkv + kvh) * head_stride;
    const u16* k1 = a.kc + ((long)b1 * a.nkv + kvh) * head_stride;
    const u16* v0 = a.vc + ((long)b0 * a.nkv + kvh) * head_stride;
    const u16* v1 = a.vc + ((long)b1 * a.nkv + kvh) * head_stride;
    // issue all K and V loads up-front (latency overlap)
    uint4 kf0[KSTEPS], kf1[KSTEPS];
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      kf0[s] = ld16(k0 + rl * D + 8 * g + 32 * s);
      kf1[s] = ld16(k1 + rl * D + 8 * g + 32 * s);
    }
    uint2 vf0[NT], vf1[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      vf0[n] = *reinterpret_cast<const uint2*>(v0 + (16 * n + rl) * BS + 4 * g);
      vf1[n] = *reinterpret_cast<const uint2*>(v1 + (16 * n + rl) * BS + 4 * g);
    }
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf0[s]), qf[s], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kf1[s]), qf[s], s1, 0, 0, 0);
    }
    // scores for row rl: keys kb + 4g + r (s0) and kb + 16 + 4g + r (s1)
    float p[8];
    float mloc = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key0 = kb + 4 * g + r, key1 = kb + 16 + 4 * g + r;
      p[r] = (key0 < row_lim && key0 < k_end) ? s0[r] * a.scale_log2 : -INFINITY;
      p[4 + r] = (key1 < row_lim && key1 < k_end) ? s1[r] * a.scale_log2 : -INFINITY;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) mloc = fmaxf(mloc, p[j]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);
    const float m_safe = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_safe);
    float lsum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { p[j] = exp2f(p[j] - m_safe); lsum += p[j]; }
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    l_run = l_run * alpha + lsum;
    m_run = m_new;
    const bf16x8 pf = __builtin_bit_cast(bf16x8, pack8(p));
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      acc[n] *= alpha;
      const uint4 vv = make_uint4(vf0[n].x, vf0[n].y, vf1[n].x, vf1[n].y);
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, acc[n], 0, 0, 0);
    }
  }

  // ---- combine the 4 waves through LDS.  acc[n][r] = O^T[dim 16n + 4g + r][row rl]
  if (g == 0) { s_m[wave][rl] = m_run; s_l[wave][rl] = l_run; }
#pragma unroll
  for (int n = 0; n < NT; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) s_o[wave][rl][16 * n + 4 * g + r] = acc[n][r];
  __syncthreads();

  for (int e = threadIdx.x; e < 16 * D; e += blockDim.x) {
    const int row = e / D, col = e % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) M = fmaxf(M, s_m[w][row]);
    const float Ms = (M == -INFINITY) ? 0.f : M;
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
      const float f = exp2f(s_m[w][row] - Ms);
      L += s_l[w][row] * f;
      O += s_o[w][row][col] * f;
    }
    const int tok = tok0 + row / G, head = kvh * G + row % G;
    if (splits == 1) {
      if (seq >= 0 && tok < qlen)
        a.out[((long)(qstart + tok) * a.nq + head) * D + col] = f2bf(L > 0.f ? O / L : 0.f);
    } else {
      const long pidx = (((long)tile * a.nkv + kvh) * splits + split) * 16 + row;
      a.part_o[pidx * D + col] = O;
      if (col == 0) { a.part_ml[pidx * 2] = M; a.part_ml[pidx * 2 + 1] = L; }
    }
  }
}

__global__ void attn_combine_kernel(AttnArgs a, int D, int splits) {
  const int tile = blockIdx.x, kvh = blockIdx.y;
  const int seq = a.tile_seq[tile];
  if (seq < 0) return;
  const int qlen = a.seq_qlen[seq], qstart = a.seq_qstart[seq], tok0 = a.tile_tok0[tile];
  for (int e = threadIdx.x; e < 16 * D; e += blockDim.x) {
    const int row = e / D, col = e % D;
    const int tok = tok0 + row / a.G, head = kvh * a.G + row % a.G;
    if (tok >= qlen) continue;
    const long base = ((long)tile * a.nkv + kvh) * splits * 16 + row;
    float M = -INFINITY;
    for (int s = 0; s < splits; ++s) M = fmaxf(M, a.part_ml[(base + s * 16) * 2]);
    const float Ms = (M == -INFINITY) ? 0.f : M;
    float L = 0.f, O = 0.f;
    for (int s = 0; s < splits; ++s) {
      const long pi = base + s * 16;
      const float f = exp2f(a.part_ml[pi * 2] - Ms);
      L += a.part_ml[pi * 2 + 1] * f;
      O += a.part_o[pi * D + col] * f;
    }
    a.out[((long)(qstart + tok) * a.nq + head) * D + col] = f2bf(L > 0.f ? O / L : 0.f);
  }
}
}  // namespace

extern "C" int dllm_paged_attention(const void* q, const void* kc, const void* vc, const int* block_tables,
                                    const int* seq_qstart, const int* seq_qlen, const int* seq_ctx,
                                    const int* tile_seq, const int* tile_tok0, void* out, float* part_o,
                                    float* part_ml, int num_tiles, int nq, int nkv, int d, int max_blocks,
                                    int splits, int causal, float scale, hipStream_t stream) {
  if (nq % nkv != 0) return -1;
  const int G = nq / nkv;
  if (16 % G != 0) return -2;
  if (splits < 1 || (splits > 1 && (!part_o || !part_ml))) return -3;
  if (num_tiles <= 0) return 0;
  AttnArgs a{(const u16*)q, (const u16*)kc, (const u16*)vc, block_tables, seq_qstart, seq_qlen, seq_ctx,
             tile_seq, tile_tok0, (u16*)out, part_o, part_ml, nq, nkv, G, max_blocks, causal, scale * LOG2E};
  dim3 grid(num_tiles, nkv, splits), block(64 * WAVES);
  switch (d) {
    case 64: hipLaunchKernelGGL(paged_attn_kernel<64>, grid, block, 0, stream, a); break;
    case 96: hipLaunchKernelGGL(paged_attn_kernel<96>, grid, block, 0, stream, a); break;
    case 128: hipLaunchKernelGGL(paged_attn_kernel<128>, grid, block, 0, stream, a); break;
    default: return -4;
  }
  if (splits > 1)
    hipLaunchKernelGGL(attn_combine_kernel, dim3(num_tiles, nkv), dim3(256), 0, stream, a, d, splits);
  return (int)hipGetLastError();
}
