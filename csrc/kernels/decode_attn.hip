// Decode attention (one query token per sequence) over the paged KV cache: wave-per-unit design.
//
// Why a separate kernel from attention.hip: decode is a pure HBM stream (every K/V byte is read
// once per step), and a 16-row-tile workgroup that interleaves 32-key chunks over 8 waves and
// merges them through LDS measured ~4.0-4.6 TB/s at TinyLlama shapes, while the bare read
// pattern reaches ~6 TB/s (scripts/exp/kvread.hip).  The gap is occupancy (112 VGPRs: 4
// waves/SIMD) and per-unit synchronisation.  Here:
//   * a WAVE owns a unit (sequence, kv head, key split): no LDS, no barriers, 4 independent
//     waves per workgroup, so a SIMD holds as many waves as its VGPRs allow and each wave keeps
//     its own 8 KB of K/V in flight;
//   * the G = nq / nkv query heads of the kv head are the MFMA columns (G <= 16): per 32-key
//     chunk S^T[32 keys][16] = K . Q^T (2 x D/32 mfma_f32_16x16x32_bf16), lane-local online
//     softmax (row = lane & 15, 2 xor-shuffles), O^T[D][16] += V^T . P^T (D/16 MFMAs) with P^T
//     taken straight from the score registers (key permutation k-slot 8g+j <-> key
//     j < 4 ? 4g+j : 16+4g+j-4, as in attention.hip: V^T is stored per block so the operand is
//     two 8-B loads per lane);
//   * block-table entries of the next chunk are loaded one trip ahead;
//   * splits (long contexts at small batch): each wave writes (m, l, O) write-through, takes a
//     ticket per (tile, kv head); the last wave of the tile merges the splits (recipe R1 of
//     common.h) — no second kernel.
// Units are (tile, kvh, split) in tile order; the engine orders tiles longest context first,
// so the dispatcher starts the longest chains first.
#include "common.h"

namespace {
constexpr int BS = 16;
constexpr float LOG2E = 1.4426950408889634f;

struct DecArgs {
  const u16* q;            // [T, nq, D]; the token of tile t is row qstart[tile_seq[t]]
  const u16* kc;           // [blocks, nkv, 16, D]
  const u16* vc;           // [blocks, nkv, D, 16]
  const int* block_tables; // [num_seqs, max_blocks]
  const int* seq_qstart;
  const int* seq_ctx;
  const int* tile_seq;     // [num_tiles] (< 0: padding tile)
  u16* out;                // [T, nq, D]
  float* part_o;           // [num_tiles * nkv * ns, 16, D]
  float* part_ml;          // [num_tiles * nkv * ns, 16, 2]
  int* counters;           // [num_tiles * nkv] zeroed; re-armed by the merging wave
  const int* split_len;    // optional device scalar: keys per split (tiles use ceil(ctx / it) <= ns splits)
  const int* items;        // optional work list (ops.decode_work_items): [0] = n, then n pairs
                           // (tile | kvh << 16, split | nsplit << 8); waves stride over it
  int num_tiles, nq, nkv, G, max_blocks, ns;
  float scale_log2;
};

// One unit: (tile, kv head, split `split` of at most `nsplit`), processed by ONE wave.
template <int D>
__device__ __forceinline__ void decode_unit(const DecArgs& a, const int tile, const int kvh, const int split,
                                            int nsplit) {
  constexpr int KSTEPS = D / 32, NT = D / 16;
  const int lane = threadIdx.x & 63;
  const int ns = a.ns;
  const int seq = a.tile_seq[tile];
  if (seq < 0) return;
  const int ctx = a.seq_ctx[seq];
  int chunk = (ctx + nsplit - 1) / nsplit;
  if (a.items == nullptr && a.split_len != nullptr) chunk = max(chunk, *a.split_len);
  chunk = (chunk + 31) & ~31;
  nsplit = max(1, (ctx + chunk - 1) / chunk);
  if (split >= nsplit) return;
  const int k_begin = split * chunk, k_end = min(ctx, k_begin + chunk);
  const int g = lane >> 4, rl = lane & 15;
  const int G = a.G;
  const int head = kvh * G + rl;
  const int qrow = a.seq_qstart[seq];

  bf16x8 qf[KSTEPS];
  {
    const u16* qp = a.q + ((long)qrow * a.nq + head) * D + 8 * g;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s)
      qf[s] = __builtin_bit_cast(bf16x8, rl < G ? ld16(qp + 32 * s) : make_uint4(0, 0, 0, 0));
  }
  f32x4 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  const int* bt = a.block_tables + (long)seq * a.max_blocks;
  const long hs = (long)BS * D;  // elements per (block, head)
  const long kvstride = (long)a.nkv * hs;
  const u16* kbase = a.kc + kvh * hs + rl * D + 8 * g;
  const u16* vbase = a.vc + kvh * hs + rl * BS + 4 * g;
  int nb0 = 0, nb1 = 0;
  if (k_begin < k_end) {
    nb0 = bt[k_begin >> 4];
    nb1 = (k_begin + 16 < k_end) ? bt[(k_begin >> 4) + 1] : nb0;
  }
  for (int kc = k_begin; kc < k_end; kc += 32) {
    const int b0 = nb0, b1 = nb1;
    uint4 kr[2][KSTEPS];
    uint2 vr[2][NT];
    const u16* k0 = kbase + b0 * kvstride;
    const u16* k1 = kbase + b1 * kvstride;
    const u16* v0 = vbase + b0 * kvstride;
    const u16* v1 = vbase + b1 * kvstride;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      kr[0][s] = ld16(k0 + 32 * s);
      kr[1][s] = ld16(k1 + 32 * s);
    }
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      vr[0][n] = *reinterpret_cast<const uint2*>(v0 + 16 * n * BS);
      vr[1][n] = *reinterpret_cast<const uint2*>(v1 + 16 * n * BS);
    }
    const int kn = kc + 32;  // next trip's block-table entries (one trip ahead)
    if (kn < k_end) {
      nb0 = bt[kn >> 4];
      nb1 = (kn + 16 < k_end) ? bt[(kn >> 4) + 1] : nb0;
    }
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kr[0][s]), qf[s], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kr[1][s]), qf[s], s1, 0, 0, 0);
    }
    float p[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      p[e] = (kc + 4 * g + e < k_end) ? s0[e] * a.scale_log2 : -INFINITY;
      p[4 + e] = (kc + 16 + 4 * g + e < k_end) ? s1[e] * a.scale_log2 : -INFINITY;
    }
    float mloc = fmaxf(fmaxf(fmaxf(p[0], p[1]), fmaxf(p[2], p[3])), fmaxf(fmaxf(p[4], p[5]), fmaxf(p[6], p[7])));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, 64));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);  // finite: key kc < k_end is valid
    const float alpha = exp2f(m_run - m_new);
    float lsum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) { p[j] = exp2f(p[j] - m_new); lsum += p[j]; }
    lsum += __shfl_xor(lsum, 16, 64);
    lsum += __shfl_xor(lsum, 32, 64);
    l_run = l_run * alpha + lsum;
    m_run = m_new;
    const bf16x8 pf = __builtin_bit_cast(bf16x8, pack8(p));
    // keys past k_end are the never-written tail of the last block (any bit pattern): P is 0 there
    // but 0 * NaN = NaN inside the MFMA, so their V^T columns are zeroed (wave-uniform test)
    if (kc + 32 > k_end) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (kc + 16 * h + 4 * g + e >= k_end) {
#pragma unroll
            for (int n = 0; n < NT; ++n) {
              uint32_t& w = (e < 2) ? vr[h][n].x : vr[h][n].y;
              w &= (e & 1) ? 0x0000ffffu : 0xffff0000u;
            }
          }
    }
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      acc[n] *= alpha;
      const uint4 vv = make_uint4(vr[0][n].x, vr[0][n].y, vr[1][n].x, vr[1][n].y);
      acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pf, acc[n], 0, 0, 0);
    }
  }
  // acc[n][e] = O^T[dim 16n + 4g + e][row rl]
  if (nsplit == 1) {
    if (rl < G) {
      const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
      u16* op = a.out + ((long)qrow * a.nq + head) * D + 4 * g;
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const uint32_t lo = (uint32_t)f2bf(acc[n][0] * inv) | ((uint32_t)f2bf(acc[n][1] * inv) << 16);
        const uint32_t hi = (uint32_t)f2bf(acc[n][2] * inv) | ((uint32_t)f2bf(acc[n][3] * inv) << 16);
        *reinterpret_cast<uint2*>(op + 16 * n) = make_uint2(lo, hi);
      }
    }
    return;
  }
  // ---- split-K: write-through partials, ticket, the last wave of (tile, kvh) merges
  const long ub = ((long)tile * a.nkv + kvh) * ns;  // first partial of this (tile, kvh)
  const unsigned obytes = (unsigned)min((long)a.num_tiles * a.nkv * ns * 16 * D * 4, 0x7fffffffL);
  const unsigned mlbytes = (unsigned)min((long)a.num_tiles * a.nkv * ns * 16 * 2 * 4, 0x7fffffffL);
  const __amdgpu_buffer_rsrc_t ro = make_rsrc(a.part_o, obytes), rml = make_rsrc(a.part_ml, mlbytes);
  if (rl < G) {
#pragma unroll
    for (int n = 0; n < NT; ++n)
      st_wt16(ro, (unsigned)((((ub + split) * 16 + rl) * D + 16 * n + 4 * g) * 4),
              make_float4(acc[n][0], acc[n][1], acc[n][2], acc[n][3]));
  }
  {  // rows (2t, 2t+1) -> one 16-B (m, l, m, l) record, written by lane 2t of group 0
    const float m1 = __shfl_xor(m_run, 1, 64), l1 = __shfl_xor(l_run, 1, 64);
    if (g == 0 && (rl & 1) == 0)
      st_wt16(rml, (unsigned)(((ub + split) * 16 + rl) * 2 * 4), make_float4(m_run, l_run, m1, l1));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int old = 0;
  int* cnt = a.counters + (long)tile * a.nkv + kvh;
  if (lane == 0) old = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0, 64);
  if (old != nsplit - 1) return;
  if (lane == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // merge: online over the splits, every lane keeps its (row rl, dims 16n + 4g + e) layout
  float M = -INFINITY, L = 0.f;
  f32x4 o[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int sp = 0; sp < nsplit; ++sp) {
    const float4 ml = ld_wt16(rml, (unsigned)(((ub + sp) * 16 + (rl & ~1)) * 2 * 4));
    const float ms = (rl & 1) ? ml.z : ml.x, ls = (rl & 1) ? ml.w : ml.y;
    if (ms == -INFINITY) continue;  // empty split (lane-uniform per row)
    const float Mn = fmaxf(M, ms);
    const float fa = exp2f(M - Mn), fb = exp2f(ms - Mn);
    L = L * fa + ls * fb;
    M = Mn;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const float4 v = ld_wt16(ro, (unsigned)((((ub + sp) * 16 + rl) * D + 16 * n + 4 * g) * 4));
      o[n][0] = o[n][0] * fa + v.x * fb;
      o[n][1] = o[n][1] * fa + v.y * fb;
      o[n][2] = o[n][2] * fa + v.z * fb;
      o[n][3] = o[n][3] * fa + v.w * fb;
    }
  }
  if (rl < G) {
    const float inv = L > 0.f ? 1.f / L : 0.f;
    u16* op = a.out + ((long)qrow * a.nq + head) * D + 4 * g;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const uint32_t lo = (uint32_t)f2bf(o[n][0] * inv) | ((uint32_t)f2bf(o[n][1] * inv) << 16);
      const uint32_t hi = (uint32_t)f2bf(o[n][2] * inv) | ((uint32_t)f2bf(o[n][3] * inv) << 16);
      *reinterpret_cast<uint2*>(op + 16 * n) = make_uint2(lo, hi);
    }
  }
}

template <int D>
__global__ void __launch_bounds__(256) decode_attn_kernel(DecArgs a) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (a.items != nullptr) {
    // persistent: every wave strides over the work list (units longest first, so the round-robin
    // approximates longest-processing-time scheduling); a fixed grid keeps graph replay valid
    // (items[0] < 0: the extended list of attention.hip, 4 ints per unit from items[4]; the
    // per-unit metadata it carries is not used here)
    const int n0 = a.items[0], n = n0 < 0 ? -n0 : n0, nw = gridDim.x * 4;
    const int* base = n0 < 0 ? a.items + 4 : a.items + 1;
    const int st = n0 < 0 ? 4 : 2;
    for (int it = wid; it < n; it += nw) {
      const int w0 = base[st * it], w1 = base[st * it + 1];
      const int tile = w0 & 0xffff, kvh = w0 >> 16, split = w1 & 0xff, nsplit = w1 >> 8;
      // a malformed unit is skipped rather than trusted (it would index past the workspaces)
      if (tile < a.num_tiles && kvh < a.nkv && nsplit <= a.ns && split < nsplit)
        decode_unit<D>(a, tile, kvh, split, nsplit);
    }
    return;
  }
  const int ns = a.ns;
  const int tile = wid / (a.nkv * ns);
  if (tile >= a.num_tiles) return;
  decode_unit<D>(a, tile, (wid / ns) % a.nkv, wid % ns, ns);
}
}  // namespace

// Host contract (checked again by csrc/bindings.cpp): G = nq / nkv in 1..16, D in {64, 96, 128},
// ns >= 1 (with a work list: the split stride of the workspaces, >= every item's nsplit); with ns > 1 part_o >= num_tiles*nkv*ns*16*D floats, part_ml >= num_tiles*nkv*ns*32
// floats and counters >= num_tiles*nkv ints (zeroed).
extern "C" int dllm_decode_attention(const void* q, const void* kc, const void* vc, const int* block_tables,
                                     const int* seq_qstart, const int* seq_ctx, const int* tile_seq, void* out,
                                     float* part_o, float* part_ml, int* counters, const int* split_len,
                                     const int* items, int grid_wgs, int num_tiles, int nq, int nkv, int d,
                                     int max_blocks, int ns, float scale, hipStream_t stream) {
  if (nkv <= 0 || nq % nkv) return -1;
  const int G = nq / nkv;
  if (G > 16) return -2;
  if (ns < 1 || (ns > 1 && (!part_o || !part_ml || !counters))) return -3;
  if (items != nullptr && grid_wgs < 1) return -5;
  if (num_tiles <= 0) return 0;
  DecArgs a{(const u16*)q, (const u16*)kc, (const u16*)vc, block_tables, seq_qstart, seq_ctx, tile_seq, (u16*)out,
            part_o, part_ml, counters, split_len, items, num_tiles, nq, nkv, G, max_blocks, ns, scale * LOG2E};
  const long units = (long)num_tiles * nkv * ns;
  const dim3 grid(items != nullptr ? (unsigned)grid_wgs : (unsigned)((units + 3) / 4));
  switch (d) {
    case 64: hipLaunchKernelGGL(decode_attn_kernel<64>, grid, dim3(256), 0, stream, a); break;
    case 96: hipLaunchKernelGGL(decode_attn_kernel<96>, grid, dim3(256), 0, stream, a); break;
    case 128: hipLaunchKernelGGL(decode_attn_kernel<128>, grid, dim3(256), 0, stream, a); break;
    default: return -4;
  }
  return (int)hipGetLastError();
}
