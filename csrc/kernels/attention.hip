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
// normalised bf16 output; otherwise it writes (m, l, O) partials, takes a ticket, and the LAST
// workgroup of the tile combines all splits in the same launch (no second kernel).
// Decode can instead pass a work list (persistent mode): a fixed grid loops over host-built
// (tile, kv head, split, nsplit) units of ~equal key counts — balanced across ragged batches
// while the launch geometry stays constant for hipGraph replay.
#include "common.h"

namespace {
constexpr int BS = 16;     // tokens per KV block
constexpr int WAVES = 4;   // LDS combine slots; a workgroup runs W = 4 or 8 waves
constexpr int COMBINE_MAXS = 16;  // split counts up to this take the parallel last-arriver combine
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
  int* counters;         // [num_tiles * nkv] zeroed; re-armed by the reducing workgroup
  const int* split_len;  // optional device scalar: keys per split (dynamic per-tile split count)
  const int* items;      // optional work list: [0] = n, then n pairs (tile | kvh << 16, split | nsplit << 8)
  int xcd_remap;         // 1: XCD-contiguous block order (prefill K/V reuse in L2)
  int nq, nkv, G, max_blocks, causal;
  int num_tiles, split_stride;  // partial-workspace geometry: [num_tiles, nkv, split_stride, 16, d]
  float scale_log2;
  // decode (qlen 1): the newest token's V, row-major [T, nkv, d] (the fused QKV GEMM's V output,
  // tgemm GemmArgs.v_rows).  The unit that owns a sequence's newest key writes it into the V^T
  // cache and patches it into its last chunk's registers, so the GEMM's V-column workgroups no
  // longer scatter 2-byte V^T stores (they were that launch's stragglers).  Null: V^T is in the
  // cache already.
  const u16* v_new;
};
// NOTE (measured, MI355X): surplus blocks are not free — a grid whose z-splits are mostly empty
// for short contexts ran 1.5-4.7x slower than the same work with z = 1, so the engine uses static
// split counts sized to the batch and keeps the dynamic split for explicit opt-in.

template <int D>
struct AttnSmem {
  float o[WAVES][16][D + 1];
  float m[WAVES][16];
  float l[WAVES][16];
  int last;
};

// One work unit: (16-row tile, kv head, split `split` of `nsplit`).  Returns with the LDS free
// for reuse only after a __syncthreads by the caller.
// Per-tile metadata: from the tile / sequence arrays, or (extended decode work list) carried in the
// work item itself, which takes two dependent global round trips off a decode unit's critical path
// (item -> tile_seq -> seq_qlen/ctx/qstart -> block table -> K/V becomes item -> block table -> K/V).
struct TileMeta {
  int seq, tok0, qlen, ctx, qstart;
};

__device__ __forceinline__ TileMeta load_tile_meta(const AttnArgs& a, int tile) {
  TileMeta t{a.tile_seq[tile], a.tile_tok0[tile], 0, 0, 0};
  if (t.seq >= 0) { t.qlen = a.seq_qlen[t.seq]; t.ctx = a.seq_ctx[t.seq]; t.qstart = a.seq_qstart[t.seq]; }
  return t;
}

template <int D, int W, bool VN>
__device__ __forceinline__ void attn_unit(const AttnArgs& a, AttnSmem<D>& sm, const int tile, const int kvh,
                                          const int split, int nsplit, const TileMeta tm) {
  constexpr int CH = 1;   // 32-key chunks per wave trip (2, and a block-table prefetch one trip ahead, measured no gain)
  constexpr int KSTEPS = D / 32;
  constexpr int NT = D / 16;
  auto& s_o = sm.o;
  auto& s_m = sm.m;
  auto& s_l = sm.l;
  const int splits = a.split_stride;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, rl = lane & 15;
  const int seq = tm.seq;
  const int G = a.G, tpt = 16 / G;
  const int tok0 = tm.tok0, qlen = tm.qlen, ctx = tm.ctx, qstart = tm.qstart;

  // this lane's row
  const int my_tok = tok0 + rl / G, my_head = kvh * G + rl % G;
  const bool row_ok = seq >= 0 && my_tok < qlen;
  const int row_lim = !row_ok ? 0 : (a.causal ? ctx - qlen + my_tok + 1 : ctx);
  int last_tok = min(tok0 + tpt, qlen) - 1;
  int kmax = (seq < 0 || last_tok < tok0) ? 0 : (a.causal ? ctx - qlen + last_tok + 1 : ctx);
  // Dynamic split-K: with a device-side split length every tile takes only as many of the
  // gridDim.z splits as its own key range needs (long contexts split, short ones run whole), so
  // one launch is balanced across a batch of very different context lengths; surplus blocks
  // leave immediately (uniform per block: split is a per-block index).
  if (a.items == nullptr && a.split_len != nullptr) {
    const int sl = max(*a.split_len, 32);
    nsplit = min(splits, max(1, (kmax + sl - 1) / sl));
    if (split >= nsplit) return;
  }
  int chunk = (kmax + nsplit - 1) / nsplit;
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
  // One register stage per 32-key chunk (a 2-stage prefetch pipeline measured SLOWER on MI355X:
  // +30 VGPRs cost a wave per SIMD, and occupancy hides the K/V latency better than ILP here).
  // (Plain local arrays in the loop body: an earlier lambda + struct form made hipcc keep part
  // of the K/V registers in scratch for some instantiations — 48-80 B/lane of scratch traffic.)

  // the newest key's V handed over row-major (AttnArgs.v_new): only the unit whose key range ends
  // at the sequence's context owns it (chunks are 32-key aligned, so no other unit reads its block)
  // (VN: a separate instantiation, so the other paths keep their register budget)
  const int vkey = (VN && seq >= 0 && qlen == 1 && k_end == kmax && k_end > k_begin) ? kmax - 1 : -1;
  for (int kb = k_begin + 32 * CH * wave; kb < k_end; kb += 32 * CH * W) {
    uint4 kr[CH][2][KSTEPS];
    uint2 vr[CH][2][NT];
    int cb0[CH], cb1[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int kc_ = kb + 32 * c;
      cb0[c] = kc_ < k_end ? bt[kc_ >> 4] : bt[kb >> 4];
      cb1[c] = (kc_ + 16 < k_end) ? bt[(kc_ >> 4) + 1] : cb0[c];
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int b0 = cb0[c], b1 = cb1[c];
      const u16* k0 = a.kc + ((long)b0 * a.nkv + kvh) * head_stride + rl * D + 8 * g;
      const u16* k1 = a.kc + ((long)b1 * a.nkv + kvh) * head_stride + rl * D + 8 * g;
      const u16* v0 = a.vc + ((long)b0 * a.nkv + kvh) * head_stride + rl * BS + 4 * g;
      const u16* v1 = a.vc + ((long)b1 * a.nkv + kvh) * head_stride + rl * BS + 4 * g;
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        kr[c][0][s] = ld16(k0 + 32 * s);
        kr[c][1][s] = ld16(k1 + 32 * s);
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        vr[c][0][n] = *reinterpret_cast<const uint2*>(v0 + 16 * n * BS);
        vr[c][1][n] = *reinterpret_cast<const uint2*>(v1 + 16 * n * BS);
      }
    }
    // the newest key's V (row-major hand-over) rides along with the trip that reads its chunk, so
    // it costs no extra round trip and holds no registers outside that trip
    uint32_t vnv[NT];
    const bool vtrip = VN && vkey >= kb && vkey < kb + 32 * CH;   // wave-uniform
    if (vtrip) {
      const u16* vp = a.v_new + ((long)qstart * a.nkv + kvh) * D + rl;
#pragma unroll
      for (int n = 0; n < NT; ++n) vnv[n] = vp[16 * n];
    }
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int kc = kb + 32 * c;
      if (kc >= k_end) break;  // wave-uniform
      f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KSTEPS; ++s) {
        s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kr[c][0][s]), qf[s], s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kr[c][1][s]), qf[s], s1, 0, 0, 0);
      }
      // scores for row rl: keys kc + 4g + r (s0) and kc + 16 + 4g + r (s1)
      float p[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int key0 = kc + 4 * g + q, key1 = kc + 16 + 4 * g + q;
        p[q] = (key0 < row_lim && key0 < k_end) ? s0[q] * a.scale_log2 : -INFINITY;
        p[4 + q] = (key1 < row_lim && key1 < k_end) ? s1[q] * a.scale_log2 : -INFINITY;
      }
      float mloc = -INFINITY;
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
      if (VN && vkey >= kc && vkey < kc + 32) {   // wave-uniform: this chunk holds the newest key
        // (every index below is a compile-time constant or a uniform branch: a runtime-indexed
        // vr[..][h][..] would put the whole K/V register stage in scratch, cdna_hip_programming.md
        // §5.4 rule 20)
        const int hv = (vkey - kc) >> 4, q = vkey & 3;
        if (g == ((vkey & 15) >> 2)) {       // lanes whose 8-byte V^T load covers that key
          u16* vcp = const_cast<u16*>(a.vc) + ((long)(hv ? cb1[c] : cb0[c]) * a.nkv + kvh) * head_stride + rl * BS +
                     (vkey & 15);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            if (h != hv) continue;
#pragma unroll
            for (int n = 0; n < NT; ++n) {
              const uint32_t nv = vnv[n];
              uint32_t wx = vr[c][h][n].x, wy = vr[c][h][n].y;
              if (q == 0) wx = (wx & 0xffff0000u) | nv;
              else if (q == 1) wx = (wx & 0x0000ffffu) | (nv << 16);
              else if (q == 2) wy = (wy & 0xffff0000u) | nv;
              else wy = (wy & 0x0000ffffu) | (nv << 16);
              vr[c][h][n].x = wx;
              vr[c][h][n].y = wy;
              vcp[16 * n * BS] = (u16)nv;   // dim 16 n + rl of the newest key, into the V^T cache
            }
          }
        }
      }
      // Keys past k_end sit in the tail of the last KV block: never written for this sequence
      // (uninitialised or stale memory, possibly NaN/Inf bit patterns).  Their P is 0, but
      // 0 * NaN = NaN inside the PV MFMA, so zero those V^T columns (wave-uniform tail test).
      if (kc + 32 > k_end) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (kc + 16 * h + 4 * g + q >= k_end) {
#pragma unroll
              for (int n = 0; n < NT; ++n) {
                uint32_t& w = (q < 2) ? vr[c][h][n].x : vr[c][h][n].y;
                w &= (q & 1) ? 0x0000ffffu : 0xffff0000u;
              }
            }
      }
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        acc[n] *= alpha;
        const uint4 vv = make_uint4(vr[c][0][n].x, vr[c][0][n].y, vr[c][1][n].x, vr[c][1][n].y);
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, acc[n], 0, 0, 0);
      }
    }
  }

  // ---- combine the waves through LDS.  acc[n][r] = O^T[dim 16n + 4g + r][row rl]
  if constexpr (W == 8) {  // waves 4..7 fold into waves 0..3 first (keeps LDS at 4 slots)
    if (wave >= WAVES) {
      if (g == 0) { s_m[wave - WAVES][rl] = m_run; s_l[wave - WAVES][rl] = l_run; }
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) s_o[wave - WAVES][rl][16 * n + 4 * g + r] = acc[n][r];
    }
    __syncthreads();
    if (wave < WAVES) {
      const float mo = s_m[wave][rl], lo = s_l[wave][rl];
      const float mn = fmaxf(m_run, mo), ms = (mn == -INFINITY) ? 0.f : mn;
      const float fa = exp2f(m_run - ms), fb = exp2f(mo - ms);
      l_run = l_run * fa + lo * fb;
      m_run = mn;
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[n][r] = acc[n][r] * fa + s_o[wave][rl][16 * n + 4 * g + r] * fb;
    }
    __syncthreads();
  }
  if (wave < WAVES) {
    if (g == 0) { s_m[wave][rl] = m_run; s_l[wave][rl] = l_run; }
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_o[wave][rl][16 * n + 4 * g + r] = acc[n][r];
  }
  __syncthreads();

  const int G_ = G;
  if (nsplit == 1) {
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
      const int tok = tok0 + row / G_, head = kvh * G_ + row % G_;
      if (seq >= 0 && tok < qlen)
        a.out[((long)(qstart + tok) * a.nq + head) * D + col] = f2bf(L > 0.f ? O / L : 0.f);
    }
    return;
  }
  // ---- split-K: write-through partials (O unnormalised in the workgroup's max frame, and per-row
  // (m, l)), ticket per (tile, kv head); the last arriver combines with sc1 loads (R1 recipe).
  const long pbase = (((long)tile * a.nkv + kvh) * splits + split) * 16;  // first row of this partial
  const unsigned obytes = (unsigned)min((long)a.num_tiles * a.nkv * splits * 16 * D * 4, 0x7fffffffL);
  const unsigned mlbytes = (unsigned)min((long)a.num_tiles * a.nkv * splits * 16 * 2 * 4, 0x7fffffffL);
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.part_o, obytes), rml = make_rsrc(a.part_ml, mlbytes);
  for (int e = threadIdx.x * 4; e < 16 * D; e += blockDim.x * 4) {
    const int row = e / D, col = e % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) M = fmaxf(M, s_m[w][row]);
    const float Ms = (M == -INFINITY) ? 0.f : M;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
      const float f = exp2f(s_m[w][row] - Ms);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] += s_o[w][row][col + j] * f;
    }
    st_wt16(ro, (unsigned)(((pbase + row) * D + col) * 4), make_float4(o[0], o[1], o[2], o[3]));
  }
  if (threadIdx.x < 8) {  // rows 2t, 2t+1: (m, l, m, l)
    float ml[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 2 * threadIdx.x + h;
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) M = fmaxf(M, s_m[w][row]);
      const float Ms = (M == -INFINITY) ? 0.f : M;
      float L = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) L += s_l[w][row] * exp2f(s_m[w][row] - Ms);
      ml[2 * h] = M;
      ml[2 * h + 1] = L;
    }
    st_wt16(rml, (unsigned)((pbase + 2 * threadIdx.x) * 2 * 4), make_float4(ml[0], ml[1], ml[2], ml[3]));
  }
  if (!ticket_last(&a.counters[tile * a.nkv + kvh], nsplit, &sm.last)) return;
  const long tbase = (((long)tile * a.nkv + kvh) * splits) * 16;
  if (nsplit <= COMBINE_MAXS) {
    // Parallel combine: every split's (m, l) pair is loaded by its own thread and every thread's
    // O partials of all splits are in flight together, so the last arriver pays ~2 memory round
    // trips instead of 3 x nsplit dependent ones (the write-through loads go past L2; at batch 1
    // that serial chain was most of a decode attention launch).  sm.o is free scratch here.
    // (Issuing the O loads before the (m, l) combine as well saves one more round trip, but the
    // 16 float4 it keeps live raised the kernel past 128 VGPRs: 4 -> 3 waves per SIMD for the
    // whole kernel and 18 % slower decode attention in the flagship profile, so it is not done.)
    float* s_pm = &sm.o[0][0][0];               // [nsplit][16] maxima, then [nsplit][16] sums
    float* s_pl = s_pm + COMBINE_MAXS * 16;
    if (threadIdx.x < 8 * nsplit) {             // thread (sp, pair): rows 2 pair, 2 pair + 1
      const int sp = threadIdx.x >> 3, pr = threadIdx.x & 7;
      const float4 q = ld_wt16(rml, (unsigned)((tbase + sp * 16 + 2 * pr) * 2 * 4));
      s_pm[sp * 16 + 2 * pr] = q.x;
      s_pl[sp * 16 + 2 * pr] = q.y;
      s_pm[sp * 16 + 2 * pr + 1] = q.z;
      s_pl[sp * 16 + 2 * pr + 1] = q.w;
    }
    __syncthreads();
    if (threadIdx.x < 16) {
      const int row = threadIdx.x;
      float M = -INFINITY;
      for (int sp = 0; sp < nsplit; ++sp) M = fmaxf(M, s_pm[sp * 16 + row]);
      const float Ms = (M == -INFINITY) ? 0.f : M;
      float L = 0.f;
      for (int sp = 0; sp < nsplit; ++sp) L += s_pl[sp * 16 + row] * exp2f(s_pm[sp * 16 + row] - Ms);
      s_m[0][row] = Ms;
      s_l[0][row] = L;
    }
    __syncthreads();
    for (int e = threadIdx.x * 4; e < 16 * D; e += blockDim.x * 4) {
      const int row = e / D, col = e % D;
      const int tok = tok0 + row / G_, head = kvh * G_ + row % G_;
      if (seq < 0 || tok >= qlen) continue;
      float4 q[COMBINE_MAXS];
#pragma unroll
      for (int sp = 0; sp < COMBINE_MAXS; ++sp)
        if (sp < nsplit) q[sp] = ld_wt16(ro, (unsigned)(((tbase + sp * 16 + row) * D + col) * 4));
      float o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sp = 0; sp < COMBINE_MAXS; ++sp) {
        if (sp < nsplit) {
          const float f = exp2f(s_pm[sp * 16 + row] - s_m[0][row]);
          o[0] += q[sp].x * f; o[1] += q[sp].y * f; o[2] += q[sp].z * f; o[3] += q[sp].w * f;
        }
      }
      const float L = s_l[0][row], inv = L > 0.f ? 1.f / L : 0.f;
      u16* dst = a.out + ((long)(qstart + tok) * a.nq + head) * D + col;
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = f2bf(o[j] * inv);
    }
    return;
  }
  if (threadIdx.x < 16) {
    const int row = threadIdx.x;
    float M = -INFINITY;
    for (int sp = 0; sp < nsplit; ++sp) {
      const float4 q = ld_wt16(rml, (unsigned)((tbase + sp * 16 + (row & ~1)) * 2 * 4));
      M = fmaxf(M, (row & 1) ? q.z : q.x);
    }
    const float Ms = (M == -INFINITY) ? 0.f : M;
    float L = 0.f;
    for (int sp = 0; sp < nsplit; ++sp) {
      const float4 q = ld_wt16(rml, (unsigned)((tbase + sp * 16 + (row & ~1)) * 2 * 4));
      const float m = (row & 1) ? q.z : q.x, l = (row & 1) ? q.w : q.y;
      L += l * exp2f(m - Ms);
    }
    s_m[0][row] = Ms;
    s_l[0][row] = L;
  }
  __syncthreads();
  for (int e = threadIdx.x * 4; e < 16 * D; e += blockDim.x * 4) {
    const int row = e / D, col = e % D;
    const int tok = tok0 + row / G_, head = kvh * G_ + row % G_;
    if (seq < 0 || tok >= qlen) continue;
    float o[4] = {0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < nsplit; ++sp) {
      const float4 mq = ld_wt16(rml, (unsigned)((tbase + sp * 16 + (row & ~1)) * 2 * 4));
      const float f = exp2f(((row & 1) ? mq.z : mq.x) - s_m[0][row]);
      const float4 q = ld_wt16(ro, (unsigned)(((tbase + sp * 16 + row) * D + col) * 4));
      o[0] += q.x * f; o[1] += q.y * f; o[2] += q.z * f; o[3] += q.w * f;
    }
    const float L = s_l[0][row], inv = L > 0.f ? 1.f / L : 0.f;
    u16* dst = a.out + ((long)(qstart + tok) * a.nq + head) * D + col;
#pragma unroll
    for (int j = 0; j < 4; ++j) dst[j] = f2bf(o[j] * inv);
  }
}

template <int D, int W, bool VN>
__global__ void __launch_bounds__(64 * W) paged_attn_kernel(AttnArgs a) {
  __shared__ AttnSmem<D> sm;
  if (a.items != nullptr) {
    // Persistent decode: a fixed grid (graph-capturable) walks a host-built list of equal-sized
    // key ranges, longest sequences first, so a batch of very different context lengths costs
    // ~(total keys / grid) per workgroup instead of the longest sequence's keys (no surplus
    // early-exit blocks, no tail of one long chain).
    // items[0] = n: pairs (tile | kvh << 16, split | nsplit << 8) from items[1]; items[0] = -n:
    // extended decode list, 16-B units from items[4]: (.., .., seq | qstart << 16, ctx), one token
    // per tile (qlen 1, tok0 0)
    const int n0 = a.items[0];
    const bool ext = n0 < 0;
    const int n = ext ? -n0 : n0;
    // units blockIdx.x, + gridDim.x, ... (an atomic-cursor fetch measured no gain: removed).
    // (One attn_unit call site: a lambda wrapper here made hipcc spill 176 B/lane to scratch.)
    int it = blockIdx.x;
    while (it < n) {
      int w0, w1;
      TileMeta tm;
      if (ext) {
        const int4 u = *reinterpret_cast<const int4*>(a.items + 4 + 4 * it);
        w0 = u.x;
        w1 = u.y;
        tm = TileMeta{u.z & 0xffff, 0, 1, u.w, (int)((unsigned)u.z >> 16)};
      } else {
        w0 = a.items[1 + 2 * it];
        w1 = a.items[2 + 2 * it];
      }
      const int tile = w0 & 0xffff, kvh = w0 >> 16, split = w1 & 0xff, nsplit = w1 >> 8;
      if (!ext) tm = load_tile_meta(a, tile < a.num_tiles ? tile : 0);
      // a malformed unit is skipped rather than trusted (it would index past the workspaces)
      if (tile < a.num_tiles && kvh < a.nkv && nsplit <= a.split_stride && split < nsplit && tm.ctx >= 0)
        attn_unit<D, W, VN>(a, sm, tile, kvh, split, nsplit, tm);
      __syncthreads();
      it += gridDim.x;
    }
    return;
  }
  // Prefill: XCD-aware block order (bijective; cdna_hip_programming.md T1): blocks b, b+8, ...
  // share an XCD (and its L2), so each XCD gets a CONTIGUOUS range of (tile, head, split) work
  // and the tiles of one sequence/head re-read the same K/V from that XCD's L2, not from HBM.
  // Decode (xcd_remap = 0): tiles carry no shared K/V; the host orders them longest context
  // first so the dispatcher starts the longest chains first and spreads them over all XCDs.
  int tile = blockIdx.x, kvh = blockIdx.y, split = blockIdx.z;
  const int splits = gridDim.z;
  if (a.xcd_remap) {
    const int nx = gridDim.x, ny = gridDim.y;
    const long n = (long)nx * ny * splits;
    const long lin = blockIdx.x + (long)nx * (blockIdx.y + (long)ny * blockIdx.z);
    const long q8 = n / 8, r8 = n % 8, xcd = lin % 8;
    const long logical = xcd * q8 + (xcd < r8 ? xcd : r8) + lin / 8;
    tile = (int)(logical % nx);
    const long rest = logical / nx;
    kvh = (int)(rest % ny);
    split = (int)(rest / ny);
  }
  attn_unit<D, W, VN>(a, sm, tile, kvh, split, splits, load_tile_meta(a, tile));
}

template <int D, int W>
void launch_attn(dim3 grid, const AttnArgs& a, hipStream_t stream) {
  // the newest-V patch costs ~10 VGPRs: only d = 64 with 8 waves keeps its occupancy (123 <= 128
  // VGPRs, 4 waves/SIMD); d = 96 / 128 would drop a wave per SIMD, so those callers keep the QKV
  // GEMM's V^T scatter (dllm_paged_attention refuses v_new for them)
  if constexpr (D == 64 && W == 8) {
    if (a.v_new != nullptr) {
      hipLaunchKernelGGL((paged_attn_kernel<D, W, true>), grid, dim3(64 * W), 0, stream, a);
      return;
    }
  }
  hipLaunchKernelGGL((paged_attn_kernel<D, W, false>), grid, dim3(64 * W), 0, stream, a);
}
}  // namespace

extern "C" int dllm_paged_attention(const void* q, const void* kc, const void* vc, const int* block_tables,
                                    const int* seq_qstart, const int* seq_qlen, const int* seq_ctx,
                                    const int* tile_seq, const int* tile_tok0, void* out, float* part_o,
                                    float* part_ml, int* counters, const int* split_len, const int* items,
                                    int grid_items, int xcd_remap, int num_tiles, int nq, int nkv, int d,
                                    int max_blocks, int splits, int causal, float scale, const void* v_new,
                                    hipStream_t stream) {
  if (nq % nkv != 0) return -1;
  const int G = nq / nkv;
  if (16 % G != 0) return -2;
  if (splits < 1 || (splits > 1 && (!part_o || !part_ml || !counters))) return -3;
  if (items != nullptr && (grid_items < 1 || xcd_remap)) return -5;
  if (num_tiles <= 0) return 0;
  AttnArgs a{(const u16*)q, (const u16*)kc, (const u16*)vc, block_tables, seq_qstart, seq_qlen, seq_ctx,
             tile_seq, tile_tok0, (u16*)out, part_o, part_ml, counters, split_len, items, xcd_remap, nq, nkv, G,
             max_blocks, causal, num_tiles, splits, scale * LOG2E, (const u16*)v_new};
  // 8 waves per workgroup when the grid alone cannot fill the CUs with memory requests
  // (decode at moderate batch: tiles x kv-heads x splits workgroups are all resident at once;
  // dynamic splitting bounds every block's key range, where 8 waves measured best)
  const long wgs = (long)num_tiles * nkv * splits;
  const int W = (items != nullptr || split_len != nullptr || wgs <= 2048) ? 8 : 4;
  if (v_new != nullptr && (d != 64 || W != 8)) return -7;
  const dim3 grid = items != nullptr ? dim3(grid_items, 1, 1) : dim3(num_tiles, nkv, splits);
switch (d) {
    case 64: W == 8 ? launch_attn<64, 8>(grid, a, stream) : launch_attn<64, 4>(grid, a, stream); break;
    case 96: W == 8 ? launch_attn<96, 8>(grid, a, stream) : launch_attn<96, 4>(grid, a, stream); break;
    case 128: W == 8 ? launch_attn<128, 8>(grid, a, stream) : launch_attn<128, 4>(grid, a, stream); break;
    default: return -4;
  }
  return (int)hipGetLastError();
}
