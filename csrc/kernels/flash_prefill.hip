// Flash-style prefill attention over the paged KV cache (causal or bidirectional), GQA-packed.
//
// Work unit: (128-row query tile, kv head).  Rows pack (token, head-in-GQA-group) exactly like the
// decode kernel (attention.hip): row r -> token tok0 + r / G, query head kvh * G + r % G, so a
// tile covers 128 / G tokens and every K/V byte it reads serves all G heads of the group.
// Four waves own 32 rows each (two 16-row MFMA fragments).  Per 32-key chunk (two 16-token KV
// blocks) the WORKGROUP stages K and V^T once into LDS and all four waves consume them — 8x less
// K/V traffic per query row than the 16-row decode-style tiles the prefill used before
// ("each 16-row tile streams the whole K/V prefix").
//
// Math per wave and chunk (the decode kernel's operand choice, cdna_hip_programming.md §3):
//   S^T[32 keys][16 rows] = K . Q^T        (A = K rows from LDS, B = Q^T fragments in registers)
//   online softmax per row (lane-local state + 2 xor-shuffles)
//   O^T[d][16 rows]      += V^T . P^T      (A = V^T from LDS, B = P^T straight from the S^T
//                                           accumulators with the key permutation of attention.hip)
// Staging: global_load_lds_dwordx4 into a 3-deep ring (counted vmcnt across a raw barrier, as in
// tgemm.hip); the K image is XOR-swizzled through the per-lane source address (rule 21) so the
// 16-lane fragment reads are conflict-free; the chunk's block-table entries are read from an LDS
// copy of the tile's block-table row (an ordinary global load there would make hipcc drain the
// ring).  Keys past the context tail (never written) get P = 0 AND a zeroed V column (0 * NaN).
#include "common.h"

typedef __attribute__((address_space(3))) void lds_void;

namespace {
constexpr float LOG2E_F = 1.4426950408889634f;
constexpr int ROWS = 128;   // query rows per workgroup
constexpr int CK = 32;      // keys per chunk
constexpr int STAGES = 3;
constexpr int MAXBT = 1024; // block-table entries staged per tile (16K-token context)

struct FlashArgs {
  const u16* q;  // [T, nq, D]
  const u16* kc; // [blocks, nkv, 16, D]
  const u16* vc; // [blocks, nkv, D, 16]
  const int* block_tables;
  const int* seq_qstart;
  const int* seq_qlen;
  const int* seq_ctx;
  const int* tile_seq;
  const int* tile_tok0;
  u16* out;
  int nq, nkv, G, max_blocks, causal;
  float scale_log2;
};

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// 16-B chunk position of chunk c of K row r in the swizzled image (conflict-free fragment reads)
template <int D>
__device__ __forceinline__ int kswz(int r, int c) {
  if constexpr (D == 128) return c ^ (r & 15);
  else return c ^ ((r >> 1) & 7);
}

template <int D>
__global__ void __launch_bounds__(256) flash_prefill_kernel(FlashArgs a) {
  constexpr int KS = D / 32;           // d-steps of S^T
  constexpr int NT = D / 16;           // dim fragments of O^T
  constexpr int KBYTES = CK * D * 2;   // K chunk (32 rows x D)
  constexpr int VBYTES = CK * D * 2;   // V^T chunk (2 blocks x D x 16)
  constexpr int STAGE = KBYTES + VBYTES;
  constexpr int GI = STAGE / 1024 / 4; // global_load_lds per wave per chunk
  static_assert(STAGE % 4096 == 0, "whole 1-KB pieces per wave");
  __shared__ __attribute__((aligned(16))) unsigned char smem[STAGES * STAGE + MAXBT * 4];
  int* s_bt = reinterpret_cast<int*>(smem + STAGES * STAGE);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, rl = lane & 15;
  const int tile = blockIdx.x, kvh = blockIdx.y;
  const int seq = a.tile_seq[tile];
  if (seq < 0) return;  // uniform
  const int G = a.G, tpt = ROWS / G;
  const int tok0 = a.tile_tok0[tile];
  const int qlen = a.seq_qlen[seq], ctx = a.seq_ctx[seq], qstart = a.seq_qstart[seq];
  const int last_tok = min(tok0 + tpt, qlen) - 1;
  if (last_tok < tok0) return;
  const int kmax = a.causal ? ctx - qlen + last_tok + 1 : ctx;
  const int nchunks = (kmax + CK - 1) / CK;
  const int* bt = a.block_tables + (long)seq * a.max_blocks;
  const int nbt = min((kmax + 15) / 16, MAXBT);
  for (int i = threadIdx.x; i < nbt; i += 256) s_bt[i] = bt[i];

  // this lane's two rows (fragments f = 0, 1 of the wave's 32 rows)
  int row_lim[2], my_tok[2], my_head[2];
  bool row_ok[2];
  bf16x8 qf[2][KS];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const int r = 32 * wave + 16 * f + rl;
    my_tok[f] = tok0 + r / G;
    my_head[f] = kvh * G + r % G;
    row_ok[f] = my_tok[f] < qlen && my_tok[f] <= last_tok;
    row_lim[f] = !row_ok[f] ? 0 : (a.causal ? ctx - qlen + my_tok[f] + 1 : ctx);
    const u16* qp = a.q + ((long)(qstart + (row_ok[f] ? my_tok[f] : tok0)) * a.nq + my_head[f]) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[f][s] = __builtin_bit_cast(bf16x8, row_ok[f] ? ld16(qp + 32 * s) : make_uint4(0, 0, 0, 0));
  }
  // keys this wave needs (causal: its last row's limit); chunks past it skip the math
  int wave_lim = 0;
  {
    const int wlast = min(tok0 + (32 * wave + 31) / G, last_tok);
    wave_lim = (tok0 + (32 * wave) / G > last_tok) ? 0 : (a.causal ? ctx - qlen + wlast + 1 : ctx);
  }
  // keys below every row's causal limit in this wave: chunks entirely under it skip the masks
  int wave_lo = min(row_lim[0], row_lim[1]);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) wave_lo = min(wave_lo, __shfl_xor(wave_lo, o, 64));
  __syncthreads();  // s_bt ready (no glds in flight yet: a plain barrier is fine)

  // staging: piece p (1 KB) of a stage; K pieces first, then V^T pieces
  const long hstride = (long)16 * D;  // elements per (block, head) in either cache
  auto issue = [&](int t) {
    unsigned char* base = smem + (t % STAGES) * STAGE;
    const int kb = t * CK;
    const int b0 = s_bt[min(kb >> 4, nbt - 1)];
    const int b1 = s_bt[min((kb >> 4) + 1, nbt - 1)];
#pragma unroll
    for (int j = 0; j < GI; ++j) {
      const int p = wave * GI + j;                    // piece index within the stage
      const int byte = p * 1024 + lane * 16;          // this lane's LDS byte within the stage
      const u16* src;
      if (byte < KBYTES) {
        const int r = byte / (2 * D), pos = (byte % (2 * D)) / 16;
        const int c = kswz<D>(r, pos);                // source chunk landing at position pos
        const int blk = (r < 16) ? b0 : b1;
        src = a.kc + ((long)blk * a.nkv + kvh) * hstride + (r & 15) * D + 8 * c;
      } else {
        const int vb = byte - KBYTES, blk = (vb < 32 * D) ? b0 : b1;
        src = a.vc + ((long)blk * a.nkv + kvh) * hstride + (vb % (32 * D)) / 2;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(base + p * 1024), 16, 0, 0);
    }
  };

  f32x4 acc[2][NT];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[f][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[2] = {-INFINITY, -INFINITY}, l_run[2] = {0.f, 0.f};

#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < nchunks) issue(t);

  for (int t = 0; t < nchunks; ++t) {
    if (t + 1 < nchunks) wait_vm<GI>(); else wait_vm<0>();
    sync_lds();
    if (t + STAGES - 1 < nchunks) issue(t + STAGES - 1);
    const int kb = t * CK;
    if (kb >= wave_lim) continue;  // wave-uniform: every row of this wave is past its causal limit
    const unsigned char* kbase = smem + (t % STAGES) * STAGE;
    const unsigned char* vbase = kbase + KBYTES;
    // S^T = K . Q^T for both row fragments; K fragments (A operand: key row 16 h + rl, dims
    // 32 s + 8 g) are read once per d-step and used by both
    f32x4 sc[2][2];
#pragma unroll
    for (int f = 0; f < 2; ++f) sc[f][0] = sc[f][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int r = 16 * h + rl, c = 4 * s + g;
        const bf16x8 kfr = *reinterpret_cast<const bf16x8*>(kbase + r * (2 * D) + (kswz<D>(r, c) << 4));
#pragma unroll
        for (int f = 0; f < 2; ++f) sc[f][h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kfr, qf[f][s], sc[f][h], 0, 0, 0);
      }
    }
    // online softmax per row fragment -> P^T (B operand of the PV product) and the rescale
    bf16x8 pf[2];
    float alpha[2];
    const bool unmasked = kb + CK <= wave_lo;  // wave-uniform: every key of the chunk is visible to every row
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      float p[8];
      if (unmasked) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          p[q] = sc[f][0][q] * a.scale_log2;
          p[4 + q] = sc[f][1][q] * a.scale_log2;
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int key0 = kb + 4 * g + q, key1 = kb + 16 + 4 * g + q;
          p[q] = (key0 < row_lim[f] && key0 < kmax) ? sc[f][0][q] * a.scale_log2 : -INFINITY;
          p[4 + q] = (key1 < row_lim[f] && key1 < kmax) ? sc[f][1][q] * a.scale_log2 : -INFINITY;
        }
      }
      float mloc = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) mloc = fmaxf(mloc, p[j]);
      mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
      mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
      const float m_new = fmaxf(m_run[f], mloc);
      const float m_safe = (m_new == -INFINITY) ? 0.f : m_new;
      alpha[f] = __builtin_amdgcn_exp2f(m_run[f] - m_safe);   // v_exp_f32 (exp2(-inf) = 0)
      float lsum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) { p[j] = __builtin_amdgcn_exp2f(p[j] - m_safe); lsum += p[j]; }
      lsum += __shfl_xor(lsum, 16, 64);
      lsum += __shfl_xor(lsum, 32, 64);
      l_run[f] = l_run[f] * alpha[f] + lsum;
      m_run[f] = m_new;
      pf[f] = __builtin_bit_cast(bf16x8, pack8(p));
    }
    // O^T += V^T . P^T; one V^T fragment (dim 16 n + rl, keys 4g..4g+3 of each block) at a time
    const bool tail = kb + CK > kmax;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const unsigned char* vp = vbase + ((16 * n + rl) * 16 + 4 * g) * 2;
      uint2 v0 = *reinterpret_cast<const uint2*>(vp);
      uint2 v1 = *reinterpret_cast<const uint2*>(vp + 32 * D);
      if (tail) {  // zero the columns of keys past the context end (never-written cache bytes)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t keep = (q & 1) ? 0x0000ffffu : 0xffff0000u;
          if (kb + 4 * g + q >= kmax) { if (q < 2) v0.x &= keep; else v0.y &= keep; }
          if (kb + 16 + 4 * g + q >= kmax) { if (q < 2) v1.x &= keep; else v1.y &= keep; }
        }
      }
      const bf16x8 vf = __builtin_bit_cast(bf16x8, make_uint4(v0.x, v0.y, v1.x, v1.y));
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        acc[f][n] *= alpha[f];
        acc[f][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[f], acc[f][n], 0, 0, 0);
      }
    }
  }

  // acc[f][n][e] = O^T[dim 16 n + 4 g + e][row rl]: 4 consecutive dims of the lane's row
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    if (!row_ok[f]) continue;
    const float inv = l_run[f] > 0.f ? 1.f / l_run[f] : 0.f;
    u16* o = a.out + ((long)(qstart + my_tok[f]) * a.nq + my_head[f]) * D + 4 * g;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const uint32_t lo = (uint32_t)f2bf(acc[f][n][0] * inv) | ((uint32_t)f2bf(acc[f][n][1] * inv) << 16);
      const uint32_t hi = (uint32_t)f2bf(acc[f][n][2] * inv) | ((uint32_t)f2bf(acc[f][n][3] * inv) << 16);
      *reinterpret_cast<uint2*>(o + 16 * n) = make_uint2(lo, hi);
    }
  }
}
}  // namespace

// Tiles: 128 / G query tokens per tile (host-built, ops.flash_tiles); grid = (tiles, nkv).
extern "C" int dllm_flash_prefill(const void* q, const void* kc, const void* vc, const int* block_tables,
                                  const int* seq_qstart, const int* seq_qlen, const int* seq_ctx, const int* tile_seq,
                                  const int* tile_tok0, void* out, int num_tiles, int nq, int nkv, int d,
                                  int max_blocks, int causal, float scale, hipStream_t stream) {
  if (nq % nkv) return -1;
  const int G = nq / nkv;
  if (ROWS % G || G > 16) return -2;
  if (num_tiles <= 0) return 0;
  FlashArgs a{(const u16*)q, (const u16*)kc, (const u16*)vc, block_tables, seq_qstart, seq_qlen, seq_ctx,
              tile_seq, tile_tok0, (u16*)out, nq, nkv, G, max_blocks, causal, scale * LOG2E_F};
  const dim3 grid(num_tiles, nkv);
  switch (d) {
    case 64: hipLaunchKernelGGL(flash_prefill_kernel<64>, grid, dim3(256), 0, stream, a); break;
    case 128: hipLaunchKernelGGL(flash_prefill_kernel<128>, grid, dim3(256), 0, stream, a); break;
    default: return -4;
  }
  return (int)hipGetLastError();
}
