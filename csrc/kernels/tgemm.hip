// LDS-tiled MFMA GEMM with fused transformer epilogues (decode batches of 16-1024 rows and
// prefill):  Y = epilogue( X[M, K] . W[N, K]^T ),  bf16 in, f32 accumulate.
//
// Why a hand-written GEMM here: at the serving operating point (M = 128-512 decode rows) the
// vendor GEMM cannot fuse, so every decoder layer paid 4 separate launch-bound kernels around its
// GEMMs (two RMSNorms, RoPE + KV scatter, SiLU*mul; profiles/r1_bench_4step_kernels_current.md).
// With the epilogues below a dense decoder layer is FIVE launches:
//
//   EPI_QKV    : y = (r . Wqkv'^T) * rinv[m]  -> RoPE on q/k -> q_out, paged K and V^T caches
//   attention
//   EPI_RESADD : r[m, n] = bf16(bf16(o . Wo^T) + r[m, n]) (residual stream, in place) and the
//                per-(n-tile, row) partial sums of r^2 for the next RMSNorm
//   EPI_SWIGLU : act = silu(g) * u with [g | u] = (r . Wgu'^T) * rinv[m]  (interleaved gate/up rows)
//   EPI_RESADD : r += act . Wd^T  (+ partial sums of squares)
//
// RMSNorm folding: rmsnorm(r) * gamma . W^T = rinv[m] * (r . (W * gamma)^T), gamma folded into the
// weight columns once at load time; rinv[m] = rsqrt(sum(r^2) / K + eps) comes from the producer
// GEMM's partial row sums (deterministic: fixed-order sum over its n-tiles, no atomics).
// Weight row orders (host side, models/llama.py): q/k head dims permuted in 32-column groups
// (dims 16g..16g+15 then d/2+16g..) so each RoPE pair (i, i + d/2) sits in two adjacent 16-column
// MFMA fragments of ONE lane; gate/up rows interleaved in 32-row groups (16 gate, 16 up) for the
// same reason.
//
// Structure (cdna_hip_programming.md §5): 4 waves (2 x 2), each wave a (BM/2) x (BN/2) tile of
// mfma_f32_16x16x32_bf16; K staged 64 deep (one 128-B line per row) through LDS by
// global_load_lds_dwordx4 (16 B per lane, lane-linear destination) into a STAGES-deep ring; the
// XOR swizzle (16-B chunk c of row r stored at chunk c ^ ((r >> 1) & 7)) is applied on the
// per-lane SOURCE address and on the ds_read_b128 address (rule 21), which makes every 16-lane
// group of a fragment read conflict-free.  Loads for the next STAGES-1 tiles stay in flight across
// the raw s_barrier (counted vmcnt; never __syncthreads in the loop: it would drain them).
// XCD-aware bijective block remap (T1): consecutive logical blocks (same weight n-tile, different
// m-tiles / k-splits) share one XCD's L2.  Optional split-K over k with the in-launch
// last-arriver combine (write-through f32 slabs + relaxed ticket, Guideline 16 R1).
#include "common.h"
#include "tgemm_args.h"

typedef __attribute__((address_space(3))) void lds_void;

namespace {
using dllm::GemmArgs;
using dllm::EPI_PLAIN;
using dllm::EPI_RESADD;
using dllm::EPI_QKV;
using dllm::EPI_SWIGLU;
constexpr int BK = 64;
constexpr int ROWB = BK * 2;  // 128 bytes per staged row

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void block_sync_lds() {
  // raw barrier: LDS accesses retired, VMEM (the in-flight global_load_lds ring) left alone
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float bfr(float x) { return bf2f(f2bf(x)); }

template <int BM, int BN, int EPI, int STAGES>
__global__ void __launch_bounds__(256) tgemm_kernel(GemmArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int FM = WM / 16, FN = WN / 16;
  constexpr int A_BYTES = BM * ROWB, STAGE_BYTES = (BM + BN) * ROWB;
  constexpr int GA = BM / 32, GB = BN / 32, G = GA + GB;  // global_load_lds per wave per stage
  constexpr int RING = STAGES * STAGE_BYTES;
  constexpr int TPR = 256 / BM;  // threads per row in the rinv reduction (2 or 4)
  // one LDS array (a second __shared__ object can make hipcc drain the ring: §5 trap 4(a))
  //   [ring][rinv partials TPR x BM][row-sum partials 2 x BM][flag]
  __shared__ __attribute__((aligned(16))) unsigned char smem[RING + TPR * BM * 4 + 2 * BM * 4 + 16];
  float* s_rsp = reinterpret_cast<float*>(smem + RING);
  float* s_red = s_rsp + TPR * BM;
  int* s_last = reinterpret_cast<int*>(s_red + 2 * BM);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int M = a.M, N = a.N, K = a.K, S = a.splits;
  const int mt = (M + BM - 1) / BM, nt = (N + BN - 1) / BN;
  const int nwg = mt * nt * S;
  // XCD-aware bijective remap (blocks b, b + 8, ... share an XCD -> contiguous logical ids)
  const int bid = blockIdx.x, q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = wgid % S, rest = wgid / S;
  const int m_tile = rest % mt, n_tile = rest / mt;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int kbeg = split * a.kchunk;
  const int nk = max(0, (min(K, kbeg + a.kchunk) - kbeg) / BK);

  // ---- row-scale prologue: the partial-sum loads are issued before the ring so they retire at
  // the ring's first wait; their sums go to LDS and are combined per row in the epilogue
  constexpr bool ROWSCALE = (EPI == EPI_QKV || EPI == EPI_SWIGLU || EPI == EPI_PLAIN);
  const bool has_rs = ROWSCALE && a.ssq_in != nullptr;
  const int rs_row = threadIdx.x % BM, rs_part = threadIdx.x / BM;
  const int rs_m = min(m0 + rs_row, M - 1);
  float ssv[8];
  if (has_rs) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s = rs_part + TPR * u;
      ssv[u] = a.ssq_in[(long)min(s, a.ssq_in_n - 1) * a.ssq_in_ld + rs_m] * (s < a.ssq_in_n ? 1.f : 0.f);
    }
  }

  // ---- staging: wave w owns ring rows [8 (w*GA + j), +8) of A and [8 (w*GB + j), +8) of B;
  // lane -> row + lane/8, LDS chunk lane%8 <- source chunk (lane%8) ^ ((row >> 1) & 7)
  const int srow = lane >> 3, spos = lane & 7;
  const u16* a_src[GA];
  const u16* b_src[GB];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int r = 8 * (wave * GA + j) + srow;
    a_src[j] = a.A + (long)min(m0 + r, M - 1) * a.lda + kbeg + 8 * (spos ^ ((r >> 1) & 7));
  }
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int r = 8 * (wave * GB + j) + srow;
    b_src[j] = a.W + (long)min(n0 + r, N - 1) * K + kbeg + 8 * (spos ^ ((r >> 1) & 7));
  }
  auto issue = [&](int t) {
    unsigned char* base = smem + (t % STAGES) * STAGE_BYTES;
    const int ko = t * BK;
#pragma unroll
    for (int j = 0; j < GA; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(a_src[j] + ko), (lds_void*)(base + (wave * GA + j) * 1024), 16,
                                       0, 0);
#pragma unroll
    for (int j = 0; j < GB; ++j)
      __builtin_amdgcn_global_load_lds((const void*)(b_src[j] + ko),
                                       (lds_void*)(base + A_BYTES + (wave * GB + j) * 1024), 16, 0, 0);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < nk) issue(t);

  if (has_rs) {
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += ssv[u];
    for (int b = rs_part + 8 * TPR; b < a.ssq_in_n; b += 8 * TPR) {  // more than 8 slots per thread
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int sl = b + TPR * u;
        s += a.ssq_in[(long)min(sl, a.ssq_in_n - 1) * a.ssq_in_ld + rs_m] * (sl < a.ssq_in_n ? 1.f : 0.f);
      }
    }
    s_rsp[rs_part * BM + rs_row] = s;  // published by the loop's first barrier (or the one below)
  }

  // ---- main loop: wait for tile t, barrier, refill the slot read at t-1, compute tile t
  for (int t = 0; t < nk; ++t) {
    if constexpr (STAGES == 3) {
      if (t + 1 < nk) wait_vm<G>(); else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    block_sync_lds();
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1);
    const unsigned char* base = smem + (t % STAGES) * STAGE_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[FM], bw[FN];
      const int c = 4 * s + (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * WM + 16 * i + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(base + r * ROWB + ((c ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * WN + 16 * j + (lane & 15);
        bw[j] = *reinterpret_cast<const bf16x8*>(base + A_BYTES + r * ROWB + ((c ^ ((r >> 1) & 7)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bw[j], acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // ring idle (every load waited), rinv partials visible

  // ---- split-K: write-through f32 slabs, ticket per output tile; the last arriver sums all
  // slabs in split order (deterministic) and runs the epilogue
  if (S > 1) {
    const int tile_id = n_tile * mt + m_tile;
    const long slab = (long)BM * BN;
    const unsigned bytes = (unsigned)min((long)mt * nt * S * slab * 4, 0x7fffffffL);
    const __amdgpu_buffer_rsrc_t pr = make_rsrc(a.part, bytes);
    const long my = ((long)tile_id * S + split) * slab;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wm * WM + 16 * i + 4 * (lane >> 4), c = wn * WN + 16 * j + (lane & 15);
        st_wt16(pr, (unsigned)((my + (long)c * BM + r) * 4),
                make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]));
      }
    if (!ticket_last(&a.counters[tile_id], S, s_last)) return;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wm * WM + 16 * i + 4 * (lane >> 4), c = wn * WN + 16 * j + (lane & 15);
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        for (int sp = 0; sp < S; ++sp) {
          const float4 q = ld_wt16(pr, (unsigned)((((long)tile_id * S + sp) * slab + (long)c * BM + r) * 4));
          v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
        }
        acc[i][j] = v;
      }
  }

  // ---- epilogue.  Lane's elements: row m0 + wm*WM + 16 i + 4 (lane>>4) + e, col n0 + wn*WN + 16 j + (lane&15)
  const int rl0 = wm * WM + 4 * (lane >> 4);
  const int cl = lane & 15;
  float rinv[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float r = 1.f;
      if (has_rs) {
        const int row = rl0 + 16 * i + e;
        float s = 0.f;
#pragma unroll
        for (int p = 0; p < TPR; ++p) s += s_rsp[p * BM + row];
        r = rsqrtf(s * a.norm_scale + a.eps);
      }
      rinv[i][e] = r;
    }

  if constexpr (EPI == EPI_PLAIN) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + rl0 + 16 * i + e;
        if (m >= M) continue;
        u16* yr = a.Y + (long)m * a.ldy;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = n0 + wn * WN + 16 * j + cl;
          if (n < N) yr[n] = f2bf(acc[i][j][e] * rinv[i][e]);
        }
      }
  } else if constexpr (EPI == EPI_RESADD) {
    float ss[FM][4];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ss[i][e] = 0.f;
        const int m = m0 + rl0 + 16 * i + e;
        if (m >= M) continue;
        u16* yr = a.Y + (long)m * a.ldy;
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int n = n0 + wn * WN + 16 * j + cl;
          if (n < N) {
            const float v = bfr(bfr(acc[i][j][e]) + bf2f(yr[n]));
            yr[n] = f2bf(v);
            ss[i][e] += v * v;
          }
        }
      }
    // row sums over the wave's 16 column lanes, then over the two column-waves through LDS
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = ss[i][e];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        if (cl == 0) s_red[wn * BM + rl0 + 16 * i + e] = v;
      }
    __syncthreads();
    if (a.ssq_out != nullptr && threadIdx.x < BM && m0 + (int)threadIdx.x < M)
      a.ssq_out[(long)n_tile * a.ssq_out_ld + m0 + threadIdx.x] = s_red[threadIdx.x] + s_red[BM + threadIdx.x];
  } else if constexpr (EPI == EPI_SWIGLU) {
    // fragment pairs (2jp, 2jp + 1) = (gate, up) of the same 16 intermediate columns
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + rl0 + 16 * i + e;
        if (m >= M) continue;
        u16* yr = a.Y + (long)m * a.ldy;
#pragma unroll
        for (int jp = 0; jp < FN / 2; ++jp) {
          const int n = n0 + wn * WN + 32 * jp;  // 32-aligned group start
          if (n >= N) continue;
          const float g = bfr(acc[i][2 * jp][e] * rinv[i][e]), u = bfr(acc[i][2 * jp + 1][e] * rinv[i][e]);
          yr[n / 2 + cl] = f2bf(silu(g) * u);
        }
      }
  } else {  // EPI_QKV
    const int d = a.d, hd = d / 2, nq = a.nq, nkv = a.nkv;
    const int qcols = nq * d, kcols = nkv * d;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + rl0 + 16 * i + e;
        if (m >= M) continue;
        const int slot = a.slots[m];
        const float* cs = a.cos_sin + (long)a.pos[m] * d;
        const long blk = slot >> 4, off = slot & 15;
#pragma unroll
        for (int jp = 0; jp < FN / 2; ++jp) {
          const int nb = n0 + wn * WN + 32 * jp;  // 32-aligned group (never straddles a head)
          if (nb >= N) continue;
          const float x1 = bfr(acc[i][2 * jp][e] * rinv[i][e]), x2 = bfr(acc[i][2 * jp + 1][e] * rinv[i][e]);
          if (nb < qcols + kcols) {
            const bool isq = nb < qcols;
            const int cc = isq ? nb : nb - qcols;
            const int head = cc / d, grp = (cc % d) >> 5;
            const int d1 = 16 * grp + cl, d2 = hd + d1;
            const float co = cs[d1], si = cs[hd + d1];
            const u16 y1 = f2bf(x1 * co - x2 * si), y2 = f2bf(x2 * co + x1 * si);
            if (isq) {
              u16* qo = a.q_out + ((long)m * nq + head) * d;
              qo[d1] = y1;
              qo[d2] = y2;
            } else if (slot >= 0) {
              u16* ko = a.kc + ((blk * nkv + head) * 16 + off) * d;
              ko[d1] = y1;
              ko[d2] = y2;
            }
          } else if (slot >= 0) {  // V: natural dim order, transposed [d][16] per block
            const int cc = nb - qcols - kcols;
            const int head = cc / d, dim = cc % d + cl;
            u16* vo = a.vc + ((blk * nkv + head) * d) * 16 + off;
            vo[(long)dim * 16] = f2bf(x1);
            vo[(long)(dim + 16) * 16] = f2bf(x2);
          }
        }
      }
  }
}

template <int BM, int BN, int EPI, int ST>
int launch_t(const GemmArgs& a, hipStream_t st) {
  const int mt = (a.M + BM - 1) / BM, nt = (a.N + BN - 1) / BN;
  hipLaunchKernelGGL((tgemm_kernel<BM, BN, EPI, ST>), dim3(mt * nt * a.splits), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

template <int BM, int BN, int EPI>
int by_stages(int stages, const GemmArgs& a, hipStream_t st) {
  return stages == 2 ? launch_t<BM, BN, EPI, 2>(a, st) : launch_t<BM, BN, EPI, 3>(a, st);
}

template <int EPI>
int by_tile(int bm, int bn, int stages, const GemmArgs& a, hipStream_t st) {
  if (bm == 64 && bn == 64) return by_stages<64, 64, EPI>(stages, a, st);
  if (bm == 64 && bn == 128) return by_stages<64, 128, EPI>(stages, a, st);
  if (bm == 128 && bn == 64) return by_stages<128, 64, EPI>(stages, a, st);
  if (bm == 128 && bn == 128) return by_stages<128, 128, EPI>(stages, a, st);
  return -20;
}

// Residual-stream helpers for the paths the GEMM epilogue cannot cover (first layer's embedding,
// tensor-parallel all-reduced outputs, MoE outputs): one wave per row, 16-B vectors.
//   res_add_ssq: r = bf16(h + r) in place (h may be null: r unchanged), ssq[m] = sum(r^2)
__global__ void __launch_bounds__(256) res_add_ssq_kernel(const u16* __restrict__ h, long ldh, u16* __restrict__ r,
                                                          long ldr, float* __restrict__ ssq, int M, int H) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  u16* rr = r + (long)row * ldr;
  const u16* hr = h ? h + (long)row * ldh : nullptr;
  float s = 0.f;
  for (int c = lane * 8; c < H; c += 512) {
    float v[8];
    unpack8(ld16(rr + c), v);
    if (hr) {
      float hv[8];
      unpack8(ld16(hr + c), hv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bfr(v[j] + hv[j]);
      st16(rr + c, pack8(v));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j] * v[j];
  }
  s = wave_sum(s);
  if (lane == 0) ssq[row] = s;
}
}  // namespace

extern "C" int dllm_res_add_ssq(const void* h, long ldh, void* r, long ldr, float* ssq, int M, int H,
                                hipStream_t stream) {
  if (H % 8 || ldr % 8 || (h && ldh % 8)) return -1;
  if (M <= 0) return 0;
  hipLaunchKernelGGL(res_add_ssq_kernel, dim3((M + 3) / 4), dim3(256), 0, stream, (const u16*)h, ldh, (u16*)r, ldr,
                     ssq, M, H);
  return (int)hipGetLastError();
}

extern "C" int dllm_tgemm_sizeof_args() { return (int)sizeof(GemmArgs); }

// Host contract (checked again by csrc/bindings.cpp): K % 64 == 0, 16-B aligned rows (lda % 8),
// splits >= 1 with kchunk % 64 == 0, part >= splits * tiles * bm * bn floats and counters >= tiles
// (zeroed) when splits > 1; QKV/SWIGLU need N % 32 == 0 (and d % 32 == 0).
extern "C" int dllm_tgemm(const void* args, int bm, int bn, int stages, int epi, hipStream_t stream) {
  const GemmArgs& a = *reinterpret_cast<const GemmArgs*>(args);
  if (a.M <= 0 || a.N <= 0) return 0;
  if (a.K % BK || a.kchunk % BK || a.kchunk <= 0 || a.splits < 1 || a.lda % 8) return -1;
  if (a.splits > 1 && (!a.part || !a.counters)) return -2;
  if ((epi == EPI_QKV || epi == EPI_SWIGLU) && (a.N % 32)) return -3;
  if (epi == EPI_QKV && (a.d % 32 || !a.q_out || !a.kc || !a.vc || !a.pos || !a.slots || !a.cos_sin)) return -4;
  if (stages != 2 && stages != 3) return -5;
  switch (epi) {
    case EPI_PLAIN: return by_tile<EPI_PLAIN>(bm, bn, stages, a, stream);
    case EPI_RESADD: return by_tile<EPI_RESADD>(bm, bn, stages, a, stream);
    case EPI_QKV: return by_tile<EPI_QKV>(bm, bn, stages, a, stream);
    case EPI_SWIGLU: return by_tile<EPI_SWIGLU>(bm, bn, stages, a, stream);
    default: return -6;
  }
}
