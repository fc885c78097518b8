// Flash-style prefill attention over the paged KV cache (causal or bidirectional), GQA-packed.
//
// Work unit: (256-row query tile, kv head).  Rows pack (token, head-in-GQA-group) exactly like the
// decode kernel (attention.hip): row r -> token tok0 + r / G, query head kvh * G + r % G, so a
// tile covers 256 / G tokens and every K/V byte it reads serves all G heads of the group.  Eight
// waves (two per SIMD) own 32 rows each.  Per 64-key chunk (four 16-token KV blocks) the WORKGROUP
// stages K and V^T once into LDS and all eight waves consume them.
// Head dims 64, 96 (Phi-3) and 128.
//
// Math per wave and chunk, on the 32x32x16 bf16 MFMA (cdna_hip_programming.md §3 operand maps):
//   S^T[32 keys][32 rows] = K . Q^T          two key blocks, D/16 k-steps each
//                                             (A = K rows from LDS, B = Q^T fragments in registers)
//   online softmax: a lane holds 16 keys of ONE query row (col = lane & 31), so the row max is an
//   in-lane fmax chain plus one exchange with lane ^ 32; exp2 via v_exp_f32 with the softmax scale
//   folded into one FMA; the O rescale is skipped when no row's max moved (exact, wave-uniform)
//   O^T[D][32 rows]      += V^T . P^T         four 16-key k-steps x D/32 dim blocks
//                                             (A = V^T rows from LDS, B = P^T straight from the
//                                             S^T accumulators, no lane movement)
// The accumulator-as-operand step needs the S^T registers 8s..8s+7 of lane half h to be 8
// CONSECUTIVE keys: the K image stores key perm(rho) in LDS row rho (bits 2 and 3 of the in-chunk
// key index swapped), which makes registers 8s+j of half h hold key 16s + 8h + j, so the V^T
// operand is one 16-B row read per k-step.
// Staging: global_load_lds_dwordx4 into a 3-deep ring (counted vmcnt across a raw barrier, as in
// tgemm.hip).  Both LDS images are XOR-swizzled through the per-lane source address so the
// 16-lane row reads are conflict-free.  The chunk's block-table entries come from an LDS copy of
// the tile's block-table row (an ordinary global load there would make hipcc drain the ring); the
// LDS image is sized at launch for the table width, so any context length runs here (re-staging a
// 16K-key window inside the loop instead spilled the d = 64 variant's issue path to scratch).
// Keys past the context tail (never written) get P = 0 AND a zeroed V element (0 * NaN).
// Grid order: consecutive workgroups (dealt round-robin to the 8 XCDs) take consecutive kv heads,
// so the tiles sharing a head's K/V meet in one XCD's L2; the last (heaviest causal) tiles go first.
#include "common.h"

typedef __attribute__((address_space(3))) void lds_void;

namespace {
constexpr float LOG2E_F = 1.4426950408889634f;
constexpr int NWAVES = 8;
constexpr int ROWS = 32 * NWAVES;  // query rows per workgroup
constexpr int CK = 64;             // keys per chunk (four cache blocks)
constexpr int STAGES = 3;

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
  int nq, nkv, G, max_blocks, causal, num_tiles;
  float scale_log2;
  // split-KV (splits > 1, for grids that would leave CUs idle: short prompts): the chunks of a
  // tile's key range are dealt to `splits` workgroups; each writes its unnormalised O and (m, l)
  // per row write-through, takes a ticket, and the LAST one combines (common.h R1 hand-off)
  int splits;
  float* part_o;    // [num_tiles * nkv * splits, ROWS, D]
  float* part_ml;   // [num_tiles * nkv * splits, ROWS, 4]: m (raw score units), l, -, -
  int* counters;    // [num_tiles * nkv], zero at launch (memset by the launcher), re-armed by the last
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

// 16-B chunk position of chunk c of K row r in the swizzled image: 16 consecutive rows reading
// one chunk hit 16 distinct 16-B bank slots (256-B / 128-B rows: XOR over the 16 / 8 chunks;
// 192-B rows (d=96, 12 chunks): the row start cycles through 4 slots, so XOR inside aligned
// groups of 4 chunks with (r >> 2) & 3)
template <int D>
__device__ __forceinline__ int kswz(int r, int c) {
  if constexpr (D == 128) return c ^ (r & 15);
  else if constexpr (D == 96) return c ^ ((r >> 2) & 3);
  else return c ^ ((r >> 1) & 7);
}
// in-chunk key held by K image row rho: bits 2 and 3 swapped (an involution)
__device__ __forceinline__ int kperm(int rho) { return (rho & ~12) | ((rho & 4) << 1) | ((rho & 8) >> 1); }
// in-block key of S^T accumulator register i of lane half h (C row (i&3) + 8(i>>2) + 4h, permuted)
__device__ __forceinline__ int keyoff(int i, int h) { return (i & 7) | (h << 3) | ((i & 8) << 1); }

// O^T += V^T . P^T for one staged chunk: k-step s = cache block s of the chunk; lane half h holds
// keys 16s + 8h + j.  Keys past the context end (never-written cache bytes) get a zeroed V element.
template <int D, int NB, bool MAYBE_TAIL = true>
__device__ __forceinline__ void pv_chunk(f32x16 (&acc)[NB], const unsigned char* vbase, const bf16x8 (&pf)[4],
                                         const int kb, const int kmax, const int rl, const int h) {
  const bool tail = MAYBE_TAIL && kb + CK > kmax;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const int dim = 32 * n + rl;
      uint4 v = ld16(vbase + s * (32 * D) + dim * 32 + ((h ^ ((dim >> 3) & 1)) << 4));
      if (tail) {
        const int k0 = kb + 16 * s + 8 * h;
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (k0 + e >= kmax) w[e >> 1] &= (e & 1) ? 0x0000ffffu : 0xffff0000u;
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
      acc[n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, v), pf[s], acc[n], 0, 0, 0);
    }
  }
}

// PIPE: the P.V product of chunk t-1 is issued between chunk t's score MFMAs and its softmax, so a
// wave's MFMA pipe works on P.V(t-1) while its VALU computes exp2 of chunk t (in the plain loop
// every MFMA of a chunk waits on that chunk's softmax).  The ring grows to 4 stages so chunk t-1's
// V^T stays resident while chunk t+2 is staged.
template <int D, int MINW, bool PIPE, bool SPLIT = false>
__global__ void __launch_bounds__(512, MINW) flash_prefill_kernel(FlashArgs a) {
  constexpr int KD = D / 16;            // k-steps of S^T
  constexpr int NB = D / 32;            // 32-dim blocks of O^T
  constexpr int KBYTES = CK * D * 2;    // K chunk: 64 rows x D
  constexpr int VBYTES = CK * D * 2;    // V^T chunk: 4 blocks x D x 16
  constexpr int STAGE = KBYTES + VBYTES;
  constexpr int NST = PIPE ? STAGES + 1 : STAGES;   // ring stages (chunks in flight ahead: STAGES - 1)
  constexpr int GI = STAGE / 1024 / NWAVES;  // 1-KB global_load_lds pieces per wave per chunk
  static_assert(STAGE % (1024 * NWAVES) == 0, "whole 1-KB pieces per wave");
  static_assert(KBYTES % 1024 == 0, "K and V^T pieces do not share a 1-KB piece");
  // ONE dynamic LDS array: [ring STAGES x STAGE][block-table row, max_blocks entries]
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int ZBYTES = PIPE ? VBYTES : 0;         // PIPE: an all-zero V^T image (first chunk's stand-in)
  unsigned char* s_zero = smem + NST * STAGE;
  int* s_bt = reinterpret_cast<int*>(smem + NST * STAGE + ZBYTES);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, rl = lane & 31;
  const int kvh = blockIdx.x % a.nkv;
  const int rest = (int)(blockIdx.x / a.nkv);
  const int nsp = SPLIT ? a.splits : 1;
  const int split = SPLIT ? rest % nsp : 0;
  const int tile = a.num_tiles - 1 - rest / nsp;
  const int seq = a.tile_seq[tile];
  if (seq < 0) return;  // uniform
  const int G = a.G, tpt = ROWS / G;
  const int tok0 = a.tile_tok0[tile];
  const int qlen = a.seq_qlen[seq], ctx = a.seq_ctx[seq], qstart = a.seq_qstart[seq];
  const int last_tok = min(tok0 + tpt, qlen) - 1;
  if (last_tok < tok0) return;
  const int kmax = a.causal ? ctx - qlen + last_tok + 1 : ctx;
  const int nchunks_all = (kmax + CK - 1) / CK;
  // this workgroup's chunks [c0, c1): per = ceil(chunks / splits), n_split non-empty splits
  const int per = (nchunks_all + nsp - 1) / nsp;
  const int n_split = per > 0 ? (nchunks_all + per - 1) / per : 1;
  if (split >= n_split) return;  // uniform: a short tile needs fewer splits
  const int c0 = split * per, c1 = min(nchunks_all, c0 + per);
  const int nchunks = c1;
  const int* bt = a.block_tables + (long)seq * a.max_blocks;
  const int nbt = min((kmax + 15) / 16, a.max_blocks);
  for (int i = threadIdx.x; i < nbt; i += 64 * NWAVES) s_bt[i] = bt[i];
  if constexpr (PIPE) {
    for (int i = threadIdx.x; i < ZBYTES / 16; i += 64 * NWAVES)
      *reinterpret_cast<uint4*>(s_zero + 16 * i) = make_uint4(0, 0, 0, 0);
  }

  // this lane's query row (both lane halves hold the same row, different keys)
  const int r = 32 * wave + rl;
  const int my_tok = tok0 + r / G, my_head = kvh * G + r % G;
  const bool row_ok = my_tok <= last_tok;
  const int row_lim = !row_ok ? 0 : (a.causal ? ctx - qlen + my_tok + 1 : ctx);
  bf16x8 qf[KD];
  {
    const u16* qp = a.q + ((long)(qstart + (row_ok ? my_tok : tok0)) * a.nq + my_head) * D + 8 * h;
#pragma unroll
    for (int s = 0; s < KD; ++s) qf[s] = __builtin_bit_cast(bf16x8, ld16(qp + 16 * s));
  }
  // keys this wave needs (causal: its last row's limit) and keys every valid row of it sees
  const int w_first = tok0 + (32 * wave) / G;
  const int w_last = min(tok0 + (32 * wave + 31) / G, last_tok);
  const int wave_lim = (w_first > last_tok) ? 0 : (a.causal ? ctx - qlen + w_last + 1 : ctx);
  const int wave_lo = a.causal ? ctx - qlen + w_first + 1 : ctx;
  __syncthreads();  // s_bt ready (no glds in flight yet: a plain barrier is fine)

  // staging: piece p (1 KB) of a stage; K pieces first, then V^T pieces
  const long hstride = (long)16 * D;  // elements per (block, head) in either cache
  auto issue = [&](int t) {
    unsigned char* base = smem + (t % NST) * STAGE;
    const int bi = (t * CK) >> 4;
#pragma unroll
    for (int j = 0; j < GI; ++j) {
      const int p = wave * GI + j;               // piece index within the stage (wave-uniform)
      const int byte = p * 1024 + lane * 16;     // this lane's LDS byte within the stage
      const u16* src;
      if (p * 1024 < KBYTES) {
        const int rho = byte / (2 * D), pos = (byte % (2 * D)) / 16;
        const int key = kperm(rho);
        const int blk = s_bt[min(bi + (key >> 4), nbt - 1)];
        src = a.kc + ((long)blk * a.nkv + kvh) * hstride + (key & 15) * D + 8 * kswz<D>(rho, pos);
      } else {
        const int vb = byte - KBYTES, b = vb / (32 * D), w = vb % (32 * D);
        const int dim = w / 32, c = ((w % 32) / 16) ^ ((dim >> 3) & 1);
        const int blk = s_bt[min(bi + b, nbt - 1)];
        src = a.vc + ((long)blk * a.nkv + kvh) * hstride + dim * 16 + 8 * c;
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(base + p * 1024), 16, 0, 0);
    }
  };

  f32x16 acc[NB];
#pragma unroll
  for (int n = 0; n < NB; ++n)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[n][i] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;  // m in raw score units (the scale is folded into exp2)
  const float cs = a.scale_log2;

#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (c0 + t < nchunks) issue(c0 + t);

  // PIPE: the previous chunk's P and V^T stage, not yet multiplied into O.  Before the first chunk
  // they are zeros (P = 0 against an all-zero V^T image: adds exactly 0), so the in-loop P.V needs no
  // branch and shares a basic block with the softmax it overlaps.  Only the context's last chunk
  // has never-written keys to mask, and its P.V always runs in the flush after the loop.
  bf16x8 pf_prev[4];
  const unsigned char* vprev = s_zero;
  int kb_prev = -CK;
  if constexpr (PIPE) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) pf_prev[i][j] = (__bf16)0.f;
  }
  for (int t = c0; t < nchunks; ++t) {
    if (t + 1 < nchunks) wait_vm<GI>(); else wait_vm<0>();
    sync_lds();
    if (t + STAGES - 1 < nchunks) issue(t + STAGES - 1);
    const int kb = t * CK;
    if (kb >= wave_lim) {  // wave-uniform: every row of this wave is past its causal limit
      if constexpr (PIPE) {  // flush before the pending chunk's stage is re-staged
        if (kb_prev >= 0) pv_chunk<D, NB>(acc, vprev, pf_prev, kb_prev, kmax, rl, h);
        kb_prev = -CK;
      }
      continue;
    }
    const unsigned char* kbase = smem + (t % NST) * STAGE;
    const unsigned char* vbase = kbase + KBYTES;

    f32x16 sc[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sc[b][i] = 0.f;
      const int rho = 32 * b + rl;
#pragma unroll
      for (int s = 0; s < KD; ++s) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kbase + rho * (2 * D) + (kswz<D>(rho, 2 * s + h) << 4));
        sc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], sc[b], 0, 0, 0);
      }
    }
    if (kb + CK > wave_lo) {  // wave-uniform: a diagonal or tail chunk -> per-key masks
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (kb + 32 * b + keyoff(i, h) >= row_lim) sc[b][i] = -INFINITY;
    }
    float mloc = sc[0][0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mloc = fmaxf(mloc, sc[0][i]);
#pragma unroll
    for (int i = 0; i < 16; ++i) mloc = fmaxf(mloc, sc[1][i]);
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);
    if constexpr (PIPE) {  // P.V of the previous chunk (never the context's tail), previous max frame
      pv_chunk<D, NB, false>(acc, vprev, pf_prev, 0, 0, rl, h);
    }
    if (__ballot(m_new != m_run)) {  // wave-uniform: some row's running max moved -> rescale
      // exp2(-inf) = 0; a split whose first chunks are all masked for a row (SPLIT) still has
      // m_run = m_new = -inf there when another row's max moves: (-inf) - (-inf) would be NaN
      const float alpha = (SPLIT && m_new == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f((m_run - m_new) * cs);
      l_run *= alpha;
#pragma unroll
      for (int n = 0; n < NB; ++n) acc[n] *= alpha;
      m_run = m_new;
    }
    const float ms = (m_run == -INFINITY) ? 0.f : m_run * cs;
    bf16x8 pf[4];
    float lsum = 0.f;
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sc[b][8 * s2 + j], cs, -ms));
          lsum += p;
          pf[2 * b + s2][j] = (__bf16)p;
        }
      }
    l_run += lsum;

    if constexpr (PIPE) {
#pragma unroll
      for (int i = 0; i < 4; ++i) pf_prev[i] = pf[i];
      vprev = vbase;
      kb_prev = kb;
    } else {
      pv_chunk<D, NB>(acc, vbase, pf, kb, kmax, rl, h);
    }
  }
  if constexpr (PIPE) {
    if (kb_prev >= 0) pv_chunk<D, NB>(acc, vprev, pf_prev, kb_prev, kmax, rl, h);
  }

  // acc[n][i] = O^T[dim 32 n + 8 (i >> 2) + 4 h + (i & 3)][row rl]
  float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  if (SPLIT && n_split > 1) {
    // split-KV: publish this split's unnormalised O and (m, l) write-through, take the ticket
    const long unit = (long)(tile * a.nkv + kvh);
    const long pbase = (unit * a.splits + split) * ROWS;     // first row of this partial
    const unsigned obytes = (unsigned)min((long)a.num_tiles * a.nkv * a.splits * ROWS * D * 4, 0x7fffffffL);
    const unsigned mlbytes = (unsigned)min((long)a.num_tiles * a.nkv * a.splits * ROWS * 4 * 4, 0x7fffffffL);
    const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.part_o, obytes), rml = make_rsrc(a.part_ml, mlbytes);
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        st_wt16(ro, (unsigned)(((pbase + r) * D + 32 * n + 8 * g + 4 * h) * 4),
                make_float4(acc[n][4 * g], acc[n][4 * g + 1], acc[n][4 * g + 2], acc[n][4 * g + 3]));
    if (h == 0) st_wt16(rml, (unsigned)((pbase + r) * 16), make_float4(m_run, l_tot, 0.f, 0.f));
    __shared__ int s_last;
    if (!ticket_last(a.counters + unit, n_split, &s_last)) return;
    // the last arriver: every split's partial of this lane's row (sc1 loads, R1) in one frame;
    // two passes over the (m, l) pairs instead of per-split arrays (dynamic indexing would spill)
    float M = -INFINITY;
    for (int q = 0; q < n_split; ++q)
      M = fmaxf(M, ld_wt16(rml, (unsigned)(((unit * a.splits + q) * ROWS + r) * 16)).x);
    const float Ms = (M == -INFINITY) ? 0.f : M * cs;
    float L = 0.f;
#pragma unroll
    for (int n = 0; n < NB; ++n)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[n][i] = 0.f;
    for (int q = 0; q < n_split; ++q) {
      const long qb = (unit * a.splits + q) * ROWS + r;
      const float4 ml = ld_wt16(rml, (unsigned)(qb * 16));
      const float f = ml.x == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ml.x * cs - Ms);
      if (f == 0.f) continue;      // a split with no key for this row contributes nothing
      L += ml.y * f;
#pragma unroll
      for (int n = 0; n < NB; ++n)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 v = ld_wt16(ro, (unsigned)((qb * D + 32 * n + 8 * g + 4 * h) * 4));
          acc[n][4 * g] += v.x * f;
          acc[n][4 * g + 1] += v.y * f;
          acc[n][4 * g + 2] += v.z * f;
          acc[n][4 * g + 3] += v.w * f;
        }
    }
    l_tot = L;
  }
  if (!row_ok) return;
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  u16* o = a.out + ((long)(qstart + my_tok) * a.nq + my_head) * D + 4 * h;
#pragma unroll
  for (int n = 0; n < NB; ++n)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const uint32_t lo = (uint32_t)f2bf(acc[n][4 * g] * inv) | ((uint32_t)f2bf(acc[n][4 * g + 1] * inv) << 16);
      const uint32_t hi = (uint32_t)f2bf(acc[n][4 * g + 2] * inv) | ((uint32_t)f2bf(acc[n][4 * g + 3] * inv) << 16);
      *reinterpret_cast<uint2*>(o + 32 * n + 8 * g) = make_uint2(lo, hi);
    }
}
}  // namespace

// Tiles: 256 / G query tokens per tile (host-built, ops.flash_tiles); 1-D grid of tiles x nkv.
// splits > 1: split-KV (part_o [num_tiles * nkv * splits, 256, d] f32, part_ml [.., 256, 4] f32,
// counters [num_tiles * nkv] int, zeroed here); splits <= 16.
extern "C" int dllm_flash_prefill(const void* q, const void* kc, const void* vc, const int* block_tables,
                                  const int* seq_qstart, const int* seq_qlen, const int* seq_ctx, const int* tile_seq,
                                  const int* tile_tok0, void* out, int num_tiles, int nq, int nkv, int d,
                                  int max_blocks, int causal, float scale, int splits, float* part_o, float* part_ml,
                                  int* counters, hipStream_t stream) {
  if (nq % nkv) return -1;
  const int G = nq / nkv;
  if (ROWS % G || G > 32) return -2;
  if (num_tiles <= 0) return 0;
  if (splits < 1 || splits > 16 || (splits > 1 && (!part_o || !part_ml || !counters))) return -5;
  // split partials are addressed through 32-bit buffer descriptors (stores past 2 GiB would be
  // dropped silently): refuse a workspace that large instead of returning wrong attention
  if (splits > 1 && (long)num_tiles * nkv * splits * ROWS * d * 4 >= (1L << 31)) return -6;
  if (splits > 1) {
    const hipError_t e = hipMemsetAsync(counters, 0, (size_t)num_tiles * nkv * sizeof(int), stream);
    if (e != hipSuccess) return (int)e;
  }
  FlashArgs a{(const u16*)q, (const u16*)kc, (const u16*)vc, block_tables, seq_qstart, seq_qlen, seq_ctx,
              tile_seq, tile_tok0, (u16*)out, nq, nkv, G, max_blocks, causal, num_tiles, scale * LOG2E_F,
              splits, part_o, part_ml, counters};
  const dim3 grid((unsigned)num_tiles * (unsigned)nkv * (unsigned)splits);
  // d=64: 4 waves per SIMD (<= 128 VGPRs, 52 KB LDS at a 16K context) = two workgroups per CU;
  // measured 1.14-1.17x over one at 2k-16k tokens (profiles/r2_flash_prefill_microbench.md)
  // d = 128 runs the software-pipelined P.V variant (4-stage ring + zero V^T image): 4-11 % faster
  // at 2k-16k tokens; at d = 64 it needs > 128 VGPRs (one workgroup per CU instead of two) and at
  // d = 96 an earlier form of it gained nothing, so they keep the plain loop
  // (profiles/r3_flash_prefill.md).
  constexpr bool pipe = true;
  auto go = [&](auto kern, int dd, bool piped) -> int {
    const size_t lds = (size_t)(piped ? STAGES + 1 : STAGES) * (2 * CK * dd * 2) + (piped ? (size_t)CK * dd * 2 : 0) +
                       ((size_t)max_blocks * 4 + 15) / 16 * 16;
    if (lds > 160 * 1024) return -3;
    if (lds > 64 * 1024) {   // past the default dynamic-LDS cap (d = 64: contexts beyond ~128K keys)
      const hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return (int)e;
    }
    hipLaunchKernelGGL(kern, grid, dim3(64 * NWAVES), lds, stream, a);
    return (int)hipGetLastError();
  };
  if (splits > 1) {   // split-KV instantiations (small grids only): 2 waves per SIMD, plain loop
    switch (d) {
      case 64: return go(flash_prefill_kernel<64, 2, false, true>, 64, false);
      case 96: return go(flash_prefill_kernel<96, 2, false, true>, 96, false);
      case 128: return go(flash_prefill_kernel<128, 2, false, true>, 128, false);
      default: return -4;
    }
  }
  switch (d) {
    case 64: return go(flash_prefill_kernel<64, 4, false>, 64, false);
    case 96: return go(flash_prefill_kernel<96, 2, false>, 96, false);
    case 128: {  // the pipelined ring + zero image need 48 KB more LDS: past ~64K keys of block table, plain loop
      const bool fits = (size_t)(STAGES + 1) * (2 * CK * 128 * 2) + (size_t)CK * 128 * 2 + ((size_t)max_blocks * 4 + 15) / 16 * 16 <= 160 * 1024;
      return pipe && fits ? go(flash_prefill_kernel<128, 2, true>, 128, true)
                          : go(flash_prefill_kernel<128, 2, false>, 128, false);
    }
    default: return -4;
  }
}
