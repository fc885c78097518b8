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
//   EPI_GELU   : y = gelu(x . W^T + bias)  (encoder FFN; PLAIN and RESADD take the same bias)
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
using dllm::EPI_GELU;
constexpr int BK = 64;
constexpr int ROWB = BK * 2;  // 128 bytes per staged row

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most r stages of ring loads (G per stage per wave) are still in flight, r <= MAXR
template <int G, int MAXR>
__device__ __forceinline__ void wait_stages(int r) {
  if constexpr (MAXR >= 6) { if (r >= 6) { wait_vm<6 * G>(); return; } }
  if constexpr (MAXR >= 5) { if (r == 5) { wait_vm<5 * G>(); return; } }
  if constexpr (MAXR >= 4) { if (r >= 4) { wait_vm<4 * G>(); return; } }
  if constexpr (MAXR >= 3) { if (r == 3) { wait_vm<3 * G>(); return; } }
  if constexpr (MAXR >= 2) { if (r == 2) { wait_vm<2 * G>(); return; } }
  if constexpr (MAXR >= 1) { if (r == 1) { wait_vm<G>(); return; } }
  wait_vm<0>();
}
__device__ __forceinline__ void block_sync_lds() {
  // raw barrier: LDS accesses retired, VMEM (the in-flight global_load_lds ring) left alone
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }
__device__ __forceinline__ float bfr(float x) { return bf2f(f2bf(x)); }
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }

// KS: 64-deep k sub-tiles per ring stage (one barrier per stage); NW: waves per k-group, laid out
// WGM (M) x NW/WGM (N), each wave a (BM/WGM) x (BN/(NW/WGM)) tile; WK: k-groups (1, or 2 with
// KS = 2): group g stages and multiplies sub-tile g of every stage, and group 1's accumulators are
// added into group 0's through LDS after the loop.  WK = 2 doubles the waves of a small output tile
// (decode-size M has few tiles: 1 wave per SIMD leaves every LDS-read -> MFMA chain exposed) and
// halves each wave's serial k chain without a global split-K combine.
// NL > 0: NL extra LOADER waves issue (and wait for) every global_load_lds of the ring while the NW
// compute waves only read LDS fragments and issue MFMAs; one raw barrier per stage hands a slot
// from the loaders (counted vmcnt before it) to the computers (lgkmcnt(0) before it) and back.
// At decode-size M a stage's fill and its MFMA chain then overlap instead of alternating inside
// each wave (profiles/r3_decode_gemm_lab.md: 5-30 % faster on the TinyLlama / Llama-3-8B decode
// projections at M = 320-512).
// BKT: k depth of a staged sub-tile, 64 (one 128-B row line) or 32 (64-B rows: half the LDS per
// stage, so the 256-row tiles of the prefill / wide-N plans fit a 4-6 stage ring; the swizzle then
// permutes the 4 chunks of a row by (row >> 2) & 3 -> {0, 2, 3, 1}, which keeps every 16-lane
// group of a fragment read on 16 distinct 16-B bank slots).
template <int BKT>
__device__ __forceinline__ int swz(int r) {
  if constexpr (BKT == 64) return (r >> 1) & 7;
  else return (0x1320 >> (4 * ((r >> 2) & 3))) & 3;
}

// MF: MFMA shape of the wave tile, 16 (mfma_f32_16x16x32_bf16, FM x FN 16 x 16 fragments) or 32
// (mfma_f32_32x32x16_bf16, (WM / 32) x (WN / 32) 32 x 32 blocks: half the MFMA instructions for the
// same tile and the SAME LDS fragment bytes per FLOP - each lane still reads one 16-B k-slice of
// one row per fragment; the swizzle stays conflict-free for the 32-row reads, see below).  With
// MF 32 every epilogue stages its bf16 values through LDS (a RoPE / SwiGLU partner column c ^ 16
// is in lane ^ 16 of the same register: one shuffle), then the common copy-out runs.
template <int BM, int BN, int EPI, int STAGES, int KS, int NW, int WK, int NL, int WGM, int BKT, int MF = 16>
__device__ __forceinline__ void tgemm_unit(const GemmArgs& a, unsigned char* smem, int M, const int S,
                                           const int SC, const int split, const int m_tile,
                                           const int n_tile, const int kbeg, const int nk) {
  // one (tile, k range) unit: the whole body of a one-unit workgroup, or one segment of a
  // stream-K workgroup (SC: slab slots per tile in the split-K workspace)
  static_assert(WK == 1 || (WK == 2 && KS == 2), "k-groups split the KS sub-tiles of a stage");
  static_assert(NL == 0 || WK == 1, "loader waves or k-groups, not both");
  constexpr int NC = NW * WK, NT = 64 * (NC + NL), NWN = NW / WGM;  // NT: threads of the block
  constexpr int WM = BM / WGM, WN = BN / NWN;
  constexpr int FM = WM / 16, FN = WN / 16;
  static_assert(FN % 2 == 0 && FM >= 1 && WM % 16 == 0 && NW % WGM == 0, "wave tile: >= 16 rows, a multiple of 32 columns");
  constexpr int RB = 2 * BKT, RPP = 1024 / RB, LPR = RB / 16;  // row bytes, rows per 1 KB piece, lanes per row
  constexpr int A_BYTES = BM * RB, SUB_BYTES = (BM + BN) * RB, STAGE_BYTES = KS * SUB_BYTES;
  constexpr int GA = NL ? 1 : BM / (RPP * NW), GB = NL ? 1 : BN / (RPP * NW);  // global_load_lds per wave per sub-tile
  constexpr int PPS = KS * (BM + BN) / RPP;                                    // 1 KB pieces per stage
  constexpr int GL = NL ? PPS / NL : 1;                                        // ... per loader wave
  static_assert(NL == 0 || PPS % NL == 0, "stage pieces must split evenly over the loader waves");
  constexpr int G = NL ? GL : (KS / WK) * (GA + GB);     // ring loads per (issuing) wave per stage
  static_assert(NL > 0 || (GA >= 1 && GB >= 1 && BM % (RPP * NW) == 0 && BN % (RPP * NW) == 0),
                "tile too small for the wave count");
  constexpr int KSTEP = BKT * KS;
  constexpr int HALVES = BKT / 32;                        // MFMA k-steps per sub-tile
  constexpr int OW = (EPI == EPI_SWIGLU) ? BN / 2 : BN;  // staged output columns per row
  constexpr int OLD = OW + 8;                             // staged row stride (bf16)
  constexpr int RING = (STAGES * STAGE_BYTES > BM * OLD * 2) ? STAGES * STAGE_BYTES : BM * OLD * 2;
  constexpr int TPR = NT >= BM ? NT / BM : 1;  // threads per row in the rinv reduction
  // one LDS array (a second __shared__ object can make hipcc drain the ring: §5 trap 4(a))
  //   [ring][rinv partials TPR x BM][row-sum partials 2 x BM][flag]
  float* s_rsp = reinterpret_cast<float*>(smem + RING);
  float* s_red = s_rsp + TPR * BM;
  int* s_last = reinterpret_cast<int*>(s_red + 2 * BM);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool loader = NL > 0 && wid >= NC;
  const int kg = loader ? 0 : wid / NW, wave = loader ? 0 : wid % NW;
  const int wm = wave / NWN, wn = wave % NWN;
  const bool fw = ((WK == 1) || kg == 0) && !loader;  // this wave owns the final accumulators
  const int N = a.N, K = a.K;
  const int mt = (a.M + BM - 1) / BM, nt = (N + BN - 1) / BN;
  int m0 = m_tile * BM;
  const int n0 = n_tile * BN;
  const u16* Wb = a.W;
  if (a.g_tiles != nullptr) {  // grouped (MoE): row tile from the device list (block-uniform exit)
    if (m_tile >= a.g_tiles[3 * a.g_max]) return;
    m0 = a.g_tiles[a.g_max + m_tile];
    M = m0 + a.g_tiles[2 * a.g_max + m_tile];
    Wb = a.W + (long)a.g_tiles[m_tile] * a.g_wstride;
  }

  // ---- row-scale prologue: the partial-sum loads are issued before the ring so they retire at
  // the ring's first wait; their sums go to LDS and are combined per row in the epilogue
  constexpr bool ROWSCALE = (EPI == EPI_QKV || EPI == EPI_SWIGLU || EPI == EPI_PLAIN);
  const bool has_rs = ROWSCALE && a.ssq_in != nullptr;
  const int rs_row = threadIdx.x % BM, rs_part = threadIdx.x / BM;
  const bool rs_on = rs_part < TPR;  // BM = 192 with 512 threads: the last 128 threads sit out
  const int rs_m = min(m0 + rs_row, M - 1);
  float ssv[8];
  if (has_rs && rs_on) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int s = rs_part + TPR * u;
      ssv[u] = a.ssq_in[(long)min(s, a.ssq_in_n - 1) * a.ssq_in_ld + rs_m] * (s < a.ssq_in_n ? 1.f : 0.f);
    }
  }

  // ---- QKV row metadata: the positions and cache slots of this lane's output rows are loaded
  // with the row-scale partials, before the ring (they retire at its first wait), so the epilogue
  // starts with them in registers: its RoPE table reads are then ONE round trip, not two dependent
  // ones (pos -> cos/sin), and the K copy-out reads its slots from LDS.  Decode-sized tiles only
  // (FM <= 2): 2 FM*4 live registers across the ring spill the large prefill tiles
  constexpr bool QPF = EPI == EPI_QKV && FM <= 2 && MF == 16;
  constexpr int QR = QPF ? FM * 4 : 1;
  int q_pos[QR], q_slot[QR];
  if constexpr (QPF) {
    if (!loader) {
      const int rlq = wm * WM + 4 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int mm = min(m0 + rlq + 16 * i + e, M - 1);
          q_pos[4 * i + e] = a.pos[mm];
          q_slot[4 * i + e] = a.slots[mm];
        }
    }
  }

  // ---- staging: wave w owns ring rows [RPP (w*GA + j), +RPP) of A and [RPP (w*GB + j), +RPP) of B;
  // lane -> row + lane/LPR, LDS chunk lane%LPR <- source chunk (lane%LPR) ^ swz(row)
  const int srow = lane / LPR, spos = lane % LPR;
  auto a_row = [&](int r) -> const u16* {  // A source of tile row r (k offset 0 of this split)
    const int row = min(m0 + r, M - 1);
    const long arow = a.g_perm != nullptr ? (long)(a.g_perm[row] / a.g_k) : (long)row;  // MoE: gathered rows
    return a.A + arow * a.lda + kbeg + 8 * (spos ^ swz<BKT>(r));
  };
  // weight source of tile row r without its k offset (row-major, or panel-major: row n of k panel
  // p at (p N + n) 64); w_koff(k) = the offset of absolute k (a multiple of BKT) from there
  const bool wp = a.w_panel != 0;
  auto b_row = [&](int r) -> const u16* {
    const long n = min(n0 + r, N - 1);
    return Wb + (wp ? n * 64 : n * K) + 8 * (spos ^ swz<BKT>(r));
  };
  auto w_koff = [&](int k) -> long { return wp ? (long)(k >> 6) * 64 * N + (k & 63) : (long)k; };
  const u16* a_src[GA];
  const u16* b_src[GB];
  const u16* l_src[GL];   // loader waves: piece lw + NL j of the stage image ([A; B] per sub-tile)
  int l_k[GL];            // ... its k offset inside a stage (sub-tile ks * BKT), -1 - that for A
  int l_off[GL];
  if constexpr (NL == 0) {
#pragma unroll
    for (int j = 0; j < GA; ++j) a_src[j] = a_row(RPP * (wave * GA + j) + srow);
#pragma unroll
    for (int j = 0; j < GB; ++j) b_src[j] = b_row(RPP * (wave * GB + j) + srow);
  } else if (loader) {
    const int lw = wid - NC;
#pragma unroll
    for (int j = 0; j < GL; ++j) {
      const int g = lw + NL * j, ks = g / ((BM + BN) / RPP), p = g % ((BM + BN) / RPP);
      const bool isa = p < BM / RPP;
      l_src[j] = isa ? a_row(RPP * p + srow) : b_row(RPP * (p - BM / RPP) + srow);
      l_k[j] = isa ? -1 - ks * BKT : ks * BKT;
      l_off[j] = ks * SUB_BYTES + p * 1024;
    }
  }
  // k-steps in the same order in every workgroup: the workgroups of an XCD that share an activation
  // or weight tile then request its lines at about the same time and hit them in the XCD's L2.  (A
  // rotated k-start per tile, tried this round, spread those requests over time: the 256 x 256
  // prefill tile's L2 hit rate fell to 11 % against hipBLASLt's 81 %, profiles/r5_decode_gemm_lab.md.)
  auto kstep = [&](int t) { return t; };
  auto issue = [&](int t) {
    const int tk = kstep(t);
    if constexpr (NL > 0) {
      unsigned char* base = smem + (t % STAGES) * STAGE_BYTES;
#pragma unroll
      for (int j = 0; j < GL; ++j) {
        const long off = l_k[j] < 0 ? (long)(tk * KSTEP - 1 - l_k[j]) : w_koff(kbeg + tk * KSTEP + l_k[j]);
        __builtin_amdgcn_global_load_lds((const void*)(l_src[j] + off), (lds_void*)(base + l_off[j]), 16, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (WK == 2 && ks != kg) continue;  // each k-group stages its own sub-tile
      unsigned char* base = smem + (t % STAGES) * STAGE_BYTES + ks * SUB_BYTES;
      const int ko = tk * KSTEP + ks * BKT;
      const long kw = w_koff(kbeg + ko);
#pragma unroll
      for (int j = 0; j < GA; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(a_src[j] + ko), (lds_void*)(base + (wave * GA + j) * 1024),
                                         16, 0, 0);
#pragma unroll
      for (int j = 0; j < GB; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(b_src[j] + kw),
                                         (lds_void*)(base + A_BYTES + (wave * GB + j) * 1024), 16, 0, 0);
    }
  };

  static_assert(MF == 16 || (MF == 32 && WM % 32 == 0 && WN % 32 == 0 && WK == 1), "32 x 32 blocks: 32-aligned wave tiles, one k-group");
  constexpr int FM32 = MF == 32 ? WM / 32 : 1, FN32 = MF == 32 ? WN / 32 : 1;
  f32x4 acc[FM][FN];   // (MF 32: unused, eliminated)
  f32x16 acc32[FM32][FN32];
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < FM32; ++i)
#pragma unroll
      for (int j = 0; j < FN32; ++j)
#pragma unroll
        for (int v = 0; v < 16; ++v) acc32[i][j][v] = 0.f;
  }

  if (NL == 0 || loader) {
#pragma unroll
    for (int t = 0; t < STAGES - 1; ++t)
      if (t < nk) issue(t);
  }

  if (has_rs && rs_on) {
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

  // ---- ping-pong main loop of the 256 x 256 tile with 32-deep k-steps (8 waves = 2 per SIMD):
  // wave group wm = 1 runs one barrier behind group 0, so on every SIMD one wave's LDS reads and
  // ring refills overlap the other wave's MFMA burst (raised priority).  Per k-step two phases
  // {memory: fragment reads (phase 0 refills the A half of the slot read at t-1, phase 1 its B half
  // and then waits for slot t+1), lgkmcnt(0), barrier, 16 MFMAs, barrier}.  Ordering (barrier k of group 0 = barrier k-1 of
  // group 1): every read of a slot retires before its wave's barrier, which both groups pass before
  // the refill of that slot is issued one step later; slot t+1 is waited for (counted vmcnt) before
  // the phase-1 barrier that every reader of it passes afterwards.
  constexpr bool PP = MF == 16 && NL == 0 && WK == 1 && KS == 1 && NW == 8 && WGM == 2 && BKT == 32 && FM == 8 &&
                      FN == 4 && STAGES >= 3;
  if constexpr (PP) {
    const bool g1 = wm == 1;
    wait_stages<G, (STAGES - 2 < 6 ? STAGES - 2 : 6)>(min(STAGES - 2, nk - 1));  // slot 0 landed
    block_sync_lds();
    if (g1) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int c = lane >> 4;
    for (int t = 0; t < nk; ++t) {
      const unsigned char* base = smem + (t % STAGES) * STAGE_BYTES;
      bf16x8 af[FM], bw[FN];
      const bool refill = t + STAGES - 1 < nk;
      const int tk_r = kstep(t + STAGES - 1);
      unsigned char* rbase = smem + ((t + STAGES - 1) % STAGES) * STAGE_BYTES;
      if (refill) {  // the slot's A half now, its B half in phase 1 (two loads per lane per phase)
#pragma unroll
        for (int j = 0; j < GA; ++j)
          __builtin_amdgcn_global_load_lds((const void*)(a_src[j] + tk_r * KSTEP),
                                           (lds_void*)(rbase + (wave * GA + j) * 1024), 16, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * WN + 16 * j + (lane & 15);
        bw[j] = *reinterpret_cast<const bf16x8*>(base + A_BYTES + r * RB + ((c ^ swz<BKT>(r)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM / 2; ++i) {
        const int r = wm * WM + 16 * i + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(base + r * RB + ((c ^ swz<BKT>(r)) << 4));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM / 2; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bw[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = FM / 2; i < FM; ++i) {
        const int r = wm * WM + 16 * i + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(base + r * RB + ((c ^ swz<BKT>(r)) << 4));
      }
      if (refill) {
        const long kw = w_koff(kbeg + tk_r * KSTEP);
#pragma unroll
        for (int j = 0; j < GB; ++j)
          __builtin_amdgcn_global_load_lds((const void*)(b_src[j] + kw),
                                           (lds_void*)(rbase + A_BYTES + (wave * GB + j) * 1024), 16, 0, 0);
      }
      if (t + 1 < nk) wait_stages<G, (STAGES - 2 < 6 ? STAGES - 2 : 6)>(min(STAGES - 2, nk - 2 - t));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = FM / 2; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bw[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (!g1) __builtin_amdgcn_s_barrier();  // both groups leave with the same barrier count
  }
  // ---- main loop: wait for tile t, barrier, refill the slot read at t-1, compute tile t
  // (NL > 0: the loader waves do the waits and refills, the compute waves only the MFMA part)
  for (int t = 0; t < (PP ? 0 : nk); ++t) {
    if (NL == 0 || loader) {
      // tile t landed once at most min(STAGES - 2, nk - 1 - t) later stages are still in flight
      wait_stages<G, (STAGES - 2 < 6 ? STAGES - 2 : 6)>(min(STAGES - 2, nk - 1 - t));
    }
    block_sync_lds();
    if (NL == 0 || loader) {
      if (t + STAGES - 1 < nk) issue(t + STAGES - 1);
    }
    if (loader) continue;
    if constexpr (MF == 32) {
      // 32 x 32 x 16 blocks: lane l holds A[row l & 31][k 8 (l >> 5) .. +7] of a 16-deep k slice and
      // B likewise (B[k][n] = W[n][k]).  A 16-lane group of ds_read_b128 reads 16 rows of one chunk:
      // with the (r >> 1) & 7 swizzle (64-deep rows) the 16-B slots 8 (r & 1) + (c ^ ((r >> 1) & 7)) of
      // those rows are 16 distinct ones, and with the 32-deep permutation 4 (r & 3) + (c ^ p((r >> 2) & 3))
      // likewise - conflict-free, as the 16 x 16 reads.
#pragma unroll
      for (int s = 0; s < (BKT / 16) * KS; ++s) {
        const unsigned char* base = smem + (t % STAGES) * STAGE_BYTES + (s / (BKT / 16)) * SUB_BYTES;
        const int c = 2 * (s % (BKT / 16)) + (lane >> 5);
        bf16x8 af[FM32], bw[FN32];
#pragma unroll
        for (int i = 0; i < FM32; ++i) {
          const int r = wm * WM + 32 * i + (lane & 31);
          af[i] = *reinterpret_cast<const bf16x8*>(base + r * RB + ((c ^ swz<BKT>(r)) << 4));
        }
#pragma unroll
        for (int j = 0; j < FN32; ++j) {
          const int r = wn * WN + 32 * j + (lane & 31);
          bw[j] = *reinterpret_cast<const bf16x8*>(base + A_BYTES + r * RB + ((c ^ swz<BKT>(r)) << 4));
        }
#pragma unroll
        for (int i = 0; i < FM32; ++i)
#pragma unroll
          for (int j = 0; j < FN32; ++j)
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bw[j], acc32[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
    for (int s = 0; s < HALVES * KS; ++s) {
      if (WK == 2 && (s / HALVES) != kg) continue;
      const unsigned char* base = smem + (t % STAGES) * STAGE_BYTES + (s / HALVES) * SUB_BYTES;
      bf16x8 af[FM], bw[FN];
      const int c = 4 * (s % HALVES) + (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm * WM + 16 * i + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(base + r * RB + ((c ^ swz<BKT>(r)) << 4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn * WN + 16 * j + (lane & 15);
        bw[j] = *reinterpret_cast<const bf16x8*>(base + A_BYTES + r * RB + ((c ^ swz<BKT>(r)) << 4));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bw[j], acc[i][j], 0, 0, 0);
    }
#if defined(DLLM_TG_SCHED) && DLLM_TG_SCHED == 1
    // lab build only (scripts/exp/gemmlab.hip): one fragment read between consecutive MFMAs, the
    // first k-step's reads up front (hipBLASLt's one-memory-op-per-MFMA-gap order)
    if constexpr (WK == 1) {
      constexpr int NMF = HALVES * KS * FM * FN, NDS = HALVES * KS * (FM + FN);
      __builtin_amdgcn_sched_group_barrier(0x100, FM + FN, 0);
#pragma unroll
      for (int q = 0; q < NMF; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (q < NDS - (FM + FN)) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
    }
#elif defined(DLLM_TG_SCHED) && DLLM_TG_SCHED == 2
    __builtin_amdgcn_iglp_opt(0);
#endif
    }
  }
  __syncthreads();  // ring idle (every load waited), rinv partials visible
  if constexpr (WK == 2) {  // k-group 1 hands its partial tile to group 0 through the idle ring
    static_assert(NW * FM * FN * 64 * 16 <= RING, "k-group exchange must fit the ring");
    float4* xch = reinterpret_cast<float4*>(smem);
    if (kg == 1) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          xch[((wave * FM + i) * FN + j) * 64 + lane] = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
    __syncthreads();
    if (kg == 0) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const float4 v = xch[((wave * FM + i) * FN + j) * 64 + lane];
          acc[i][j][0] += v.x; acc[i][j][1] += v.y; acc[i][j][2] += v.z; acc[i][j][3] += v.w;
        }
    }
    __syncthreads();  // the ring is reused by the epilogue staging
  }

  // ---- split-K: write-through f32 slabs, ticket per output tile; the last arriver sums all
  // slabs in split order (deterministic) and runs the epilogue.  Slab layout (either MF):
  // column-major [BN][BM] f32, four consecutive rows per 16-B store
  if constexpr (MF == 32) {
    if (S > 1) {
      const int tile_id = n_tile * mt + m_tile;
      const long slab = (long)BM * BN;
      const unsigned bytes = (unsigned)min((long)mt * nt * SC * slab * 4, 0x7fffffffL);
      const __amdgpu_buffer_rsrc_t pr = make_rsrc(a.part, bytes);
      const long my = ((long)tile_id * SC + split) * slab;
      if (fw) {
#pragma unroll
        for (int i = 0; i < FM32; ++i)
#pragma unroll
          for (int j = 0; j < FN32; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int r = wm * WM + 32 * i + 8 * q + 4 * (lane >> 5), c = wn * WN + 32 * j + (lane & 31);
              st_wt16(pr, (unsigned)((my + (long)c * BM + r) * 4),
                      make_float4(acc32[i][j][4 * q], acc32[i][j][4 * q + 1], acc32[i][j][4 * q + 2], acc32[i][j][4 * q + 3]));
            }
      }
      if (!ticket_last(&a.counters[tile_id], S, s_last)) return;
      if (fw) {
#pragma unroll
        for (int i = 0; i < FM32; ++i)
#pragma unroll
          for (int j = 0; j < FN32; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int r = wm * WM + 32 * i + 8 * q + 4 * (lane >> 5), c = wn * WN + 32 * j + (lane & 31);
              float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
              for (int sp = 0; sp < S; ++sp) {
                const float4 x = ld_wt16(pr, (unsigned)((((long)tile_id * SC + sp) * slab + (long)c * BM + r) * 4));
                v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w;
              }
              acc32[i][j][4 * q] = v.x; acc32[i][j][4 * q + 1] = v.y;
              acc32[i][j][4 * q + 2] = v.z; acc32[i][j][4 * q + 3] = v.w;
            }
      }
    }
  } else if (S > 1) {
    const int tile_id = n_tile * mt + m_tile;
    const long slab = (long)BM * BN;
    const unsigned bytes = (unsigned)min((long)mt * nt * SC * slab * 4, 0x7fffffffL);
    const __amdgpu_buffer_rsrc_t pr = make_rsrc(a.part, bytes);
    const long my = ((long)tile_id * SC + split) * slab;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        if (!fw) continue;
        const int r = wm * WM + 16 * i + 4 * (lane >> 4), c = wn * WN + 16 * j + (lane & 15);
        st_wt16(pr, (unsigned)((my + (long)c * BM + r) * 4),
                make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]));
      }
    if (!ticket_last(&a.counters[tile_id], S, s_last)) return;
    if (fw && FM * FN > 16) {   // big wave tiles: no registers to spare for a slab's fragments
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int r = wm * WM + 16 * i + 4 * (lane >> 4), c = wn * WN + 16 * j + (lane & 15);
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          for (int sp = 0; sp < S; ++sp) {
            const float4 q = ld_wt16(pr, (unsigned)((((long)tile_id * SC + sp) * slab + (long)c * BM + r) * 4));
            v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
          }
          acc[i][j] = v;
        }
    } else if (fw) {
      // one round trip per split: every fragment of a slab is loaded before any is added
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int sp = 0; sp < S; ++sp) {
        float4 q[FM][FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int r = wm * WM + 16 * i + 4 * (lane >> 4), c = wn * WN + 16 * j + (lane & 15);
            q[i][j] = ld_wt16(pr, (unsigned)((((long)tile_id * SC + sp) * slab + (long)c * BM + r) * 4));
          }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            acc[i][j][0] += q[i][j].x; acc[i][j][1] += q[i][j].y; acc[i][j][2] += q[i][j].z; acc[i][j][3] += q[i][j].w;
          }
      }
    }
  }

  // ---- epilogue.  Lane's elements: row m0 + wm*WM + 16 i + 4 (lane>>4) + e, col n0 + wn*WN + 16 j + (lane&15)
  const int rl0 = wm * WM + 4 * (lane >> 4);
  const int cl = lane & 15;
  float rinv[FM][4];
#pragma unroll
  for (int i = 0; i < (MF == 16 ? FM : 0); ++i)
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

  // Output staging: every epilogue writes its bf16 results into an LDS image of the tile
  // ([BM][OW + 8] bf16, row pad = one 16-B slot against bank conflicts; the ring is idle now)
  // and the block then copies it out as 16-B row vectors, so global stores are full-width and
  // coalesced instead of 2-B scattered lane stores (RESADD reads the residual the same way).
  static_assert(BM * OLD * 2 <= RING, "output stage must fit the ring");
  u16* so = reinterpret_cast<u16*>(smem);
  const bool full_n = n0 + BN <= N;  // (N % 8 == 0 is required on the host side for vector stores)

  if constexpr (MF == 32) {
    // 32 x 32 blocks: element v of acc32[i][j] is row wm*WM + 32 i + (v & 3) + 8 (v >> 2) + 4 (lane >> 5),
    // column wn*WN + 32 j + (lane & 31).  Every epilogue value goes to the LDS image `so` here (the
    // partner column c ^ 16 of a RoPE / SwiGLU pair sits in lane ^ 16, same rows); the copy-out
    // passes below are the MF-independent ones.
    const int lc = lane & 31, c16 = lane & 15, hi = (lane >> 4) & 1;
    float bcol[FN32];
#pragma unroll
    for (int j = 0; j < FN32; ++j) {
      const int n = n0 + wn * WN + 32 * j + lc;
      bcol[j] = (EPI != EPI_SWIGLU && EPI != EPI_QKV && a.bias != nullptr && n < N) ? bf2f(a.bias[n]) : 0.f;
    }
    if (fw) {
#pragma unroll
      for (int i = 0; i < FM32; ++i)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int rl = wm * WM + 32 * i + (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5);
          float ri = 1.f;
          if (has_rs) {
            float sum = 0.f;
#pragma unroll
            for (int p = 0; p < TPR; ++p) sum += s_rsp[p * BM + rl];
            ri = rsqrtf(sum * a.norm_scale + a.eps);
          }
          if constexpr (EPI == EPI_QKV) {
            const int d = a.d, hd = d / 2, nkv = a.nkv, qcols = a.nq * d, kcols = nkv * d;
            const int m = m0 + rl, mq = min(m, M - 1);
            const int slot = a.slots[mq];
            if (wn == 0 && lc == 0) reinterpret_cast<int*>(s_red)[rl] = slot;
            const float* cs = a.cos_sin + (long)a.pos[mq] * d;
#pragma unroll
            for (int j = 0; j < FN32; ++j) {
              const int cb = wn * WN + 32 * j, nb = n0 + cb;
              const float xs = bfr(acc32[i][j][v] * ri);
              const float xp = __shfl_xor(xs, 16, 64);
              if (nb >= N) continue;   // wave-uniform
              if (nb < qcols + kcols) {
                const int cc = nb < qcols ? nb : nb - qcols;
                const int d1 = 16 * ((cc % d) >> 5) + c16;
                const float co = cs[d1], si = cs[hd + d1];
                // first half (x1 = own, x2 = partner): x1 co - x2 si; second half: x2 co + x1 si
                so[rl * OLD + cb + lc] = f2bf(hi ? xs * co + xp * si : xs * co - xp * si);
              } else if (a.v_rows != nullptr) {
                so[rl * OLD + cb + lc] = f2bf(xs);
              } else if (m < M && slot >= 0) {
                const int cc = nb - qcols - kcols;
                u16* vo = a.vc + (((long)(slot >> 4) * nkv + cc / d) * d) * 16 + (slot & 15);
                vo[(long)(cc % d + lc) * 16] = f2bf(xs);
              }
            }
          } else if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
            for (int j = 0; j < FN32; ++j) {
              const float xs = bfr(acc32[i][j][v] * ri);
              const float xp = __shfl_xor(xs, 16, 64);
              if (!hi) so[rl * OLD + (wn * WN + 32 * j) / 2 + c16] = f2bf(silu(xs) * xp);
            }
          } else {
#pragma unroll
            for (int j = 0; j < FN32; ++j) {
              float x = acc32[i][j][v] * ri + bcol[j];
              if constexpr (EPI == EPI_GELU) x = gelu_erf(bfr(x));
              so[rl * OLD + wn * WN + 32 * j + lc] = f2bf(x);
            }
          }
        }
    }
  }

  if constexpr (EPI == EPI_QKV) {
    // RoPE in registers (pairs in adjacent fragments of one lane), V written straight from the
    // registers (transposed cache layout: no row vectors to form), q/k staged.
    const int d = a.d, hd = d / 2, nq = a.nq, nkv = a.nkv;
    const int qcols = nq * d, kcols = nkv * d;
    int* s_slot = reinterpret_cast<int*>(s_red);   // [BM] cache slot per tile row (copy-out)
    if (fw && MF == 16) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rl = rl0 + 16 * i + e, m = m0 + rl;
        const int mq = min(m, M - 1);
        const int slot = QPF ? q_slot[(4 * i + e) % QR] : a.slots[mq];
        if (wn == 0 && cl == 0) s_slot[rl] = slot;
        const float* cs = a.cos_sin + (long)(QPF ? q_pos[(4 * i + e) % QR] : a.pos[mq]) * d;
        const long blk = slot >> 4, off = slot & 15;
#pragma unroll
        for (int jp = 0; jp < FN / 2; ++jp) {
          const int cb = wn * WN + 32 * jp;  // tile column of this 32-aligned group
          const int nb = n0 + cb;
          if (nb >= N) continue;
          const float x1 = bfr(acc[i][2 * jp][e] * rinv[i][e]), x2 = bfr(acc[i][2 * jp + 1][e] * rinv[i][e]);
          if (nb < qcols + kcols) {
            const int cc = nb < qcols ? nb : nb - qcols;
            const int d1 = 16 * ((cc % d) >> 5) + cl;
            const float co = cs[d1], si = cs[hd + d1];
            so[rl * OLD + cb + cl] = f2bf(x1 * co - x2 * si);
            so[rl * OLD + cb + 16 + cl] = f2bf(x2 * co + x1 * si);
          } else if (a.v_rows != nullptr) {
            // V staged like q/k and copied out as 16-B row vectors (natural dim order)
            so[rl * OLD + cb + cl] = f2bf(x1);
            so[rl * OLD + cb + 16 + cl] = f2bf(x2);
          } else if (m < M && slot >= 0) {
            // V^T cache directly: 2-byte stores 32 B apart (the slow form: a workgroup holding
            // V columns takes several us longer than its q/k neighbours at decode batch sizes)
            const int cc = nb - qcols - kcols;
            const int head = cc / d, dim = cc % d + cl;
            u16* vo = a.vc + ((blk * nkv + head) * d) * 16 + off;
            vo[(long)dim * 16] = f2bf(x1);
            vo[(long)(dim + 16) * 16] = f2bf(x2);
          }
        }
      }
    }
    __syncthreads();
    // copy-out of q/k: an 8-column chunk of a 16-column half-group is 8 consecutive natural dims
    for (int e = threadIdx.x; e < BM * (BN / 8); e += NT) {
      const int rl = e / (BN / 8), c0 = (e % (BN / 8)) * 8;
      const int m = m0 + rl, n = n0 + c0;
      if (m >= M || n >= N) continue;
      if (n >= qcols + kcols) {
        if (a.v_rows != nullptr) st16(a.v_rows + (long)m * a.v_ld + (n - qcols - kcols), *reinterpret_cast<const uint4*>(so + rl * OLD + c0));
        continue;
      }
      const bool isq = n < qcols;
      const int cc = isq ? n : n - qcols;
      const int head = cc / d, o = cc % d;
      const int dim = ((o & 31) >> 4) * hd + 16 * (o >> 5) + (o & 15);
      const uint4 v = *reinterpret_cast<const uint4*>(so + rl * OLD + c0);
      if (isq) {
        st16(a.q_out + ((long)m * nq + head) * d + dim, v);
      } else {
        const int slot = s_slot[rl];
        if (slot >= 0) st16(a.kc + (((long)(slot >> 4) * nkv + head) * 16 + (slot & 15)) * d + dim, v);
      }
    }
    return;
  } else {
    // bias (encoder layers): one value per lane column, hoisted out of the row loop
    float bcol[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + wn * WN + 16 * j + cl;
      bcol[j] = (MF == 16 && EPI != EPI_SWIGLU && a.bias != nullptr && n < N) ? bf2f(a.bias[n]) : 0.f;
    }
    if (fw && MF == 16) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rl = rl0 + 16 * i + e;
        if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
          for (int jp = 0; jp < FN / 2; ++jp) {
            const float g = bfr(acc[i][2 * jp][e] * rinv[i][e]), u = bfr(acc[i][2 * jp + 1][e] * rinv[i][e]);
            so[rl * OLD + (wn * WN + 32 * jp) / 2 + cl] = f2bf(silu(g) * u);
          }
        } else {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            float v = acc[i][j][e] * rinv[i][e] + bcol[j];
            if constexpr (EPI == EPI_GELU) v = gelu_erf(bfr(v));  // GELU of the bf16 linear output
            so[rl * OLD + wn * WN + 16 * j + cl] = f2bf(v);
          }
        }
      }
    }
    __syncthreads();
  }

  constexpr int CPR = OW / 8;  // 16-B chunks per staged row
  const int ncol0 = (EPI == EPI_SWIGLU) ? n0 / 2 : n0;
  const int nlim = (EPI == EPI_SWIGLU) ? N / 2 : N;
  if constexpr (EPI == EPI_RESADD) {
    // each thread owns chunks of one row per pass; CPR consecutive lanes share a row -> the row's
    // sum of squares is reduced with shuffles and written once per (n-tile, row)
    constexpr int RPP = NT / CPR;  // rows per pass (need not divide BM with loader waves)
    const int c0 = (threadIdx.x % CPR) * 8;
    for (int r0 = 0; r0 < BM; r0 += RPP) {
      const int rl = r0 + threadIdx.x / CPR, n = ncol0 + c0;
      const int m = rl < BM ? m0 + rl : M;  // past the tile: not this workgroup's rows
      float ss = 0.f;
      if (m < M && (full_n || n < nlim)) {
        u16* yp = a.Y + (long)m * a.ldy + n;
        float h[8], r[8];
        unpack8(*reinterpret_cast<const uint4*>(so + rl * OLD + c0), h);
        unpack8(ld16(yp), r);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          r[j] = bfr(h[j] + r[j]);
          ss += r[j] * r[j];
        }
        st16(yp, pack8(r));
      }
#pragma unroll
      for (int o = 1; o < CPR; o <<= 1) ss += __shfl_xor(ss, o, 64);
      if (a.ssq_out != nullptr && threadIdx.x % CPR == 0 && m < M) a.ssq_out[(long)n_tile * a.ssq_out_ld + m] = ss;
    }
  } else {
    for (int e = threadIdx.x; e < BM * CPR; e += NT) {
      const int rl = e / CPR, c0 = (e % CPR) * 8, m = m0 + rl, n = ncol0 + c0;
      if (m < M && (full_n || n < nlim))
        st16(a.Y + (long)m * a.ldy + n, *reinterpret_cast<const uint4*>(so + rl * OLD + c0));
    }
  }
}

template <int BM, int BN, int EPI, int STAGES, int KS, int NW, int WK = 1, int NL = 0, int WGM = 2, bool SK = false,
          int BKT = 64, int MF = 16>
__global__ void __launch_bounds__(64 * (NW * WK + NL)) tgemm_kernel(GemmArgs a) {
  static_assert(WK == 1 || (WK == 2 && KS == 2), "k-groups split the KS sub-tiles of a stage");
  static_assert(NL == 0 || WK == 1, "loader waves or k-groups, not both");
  constexpr int NC = NW * WK, NT = 64 * (NC + NL), NWN = NW / WGM;  // NT: threads of the block
  constexpr int WM = BM / WGM, WN = BN / NWN;
  constexpr int FM = WM / 16, FN = WN / 16;
  static_assert(FN % 2 == 0 && FM >= 1 && WM % 16 == 0 && NW % WGM == 0, "wave tile: >= 16 rows, a multiple of 32 columns");
  constexpr int STAGE_BYTES = KS * (BM + BN) * 2 * BKT;
  constexpr int KSTEP = BKT * KS;
  constexpr int OW = (EPI == EPI_SWIGLU) ? BN / 2 : BN;  // staged output columns per row
  constexpr int OLD = OW + 8;                             // staged row stride (bf16)
  constexpr int RING = (STAGES * STAGE_BYTES > BM * OLD * 2) ? STAGES * STAGE_BYTES : BM * OLD * 2;
  constexpr int TPR = NT >= BM ? NT / BM : 1;  // threads per row in the rinv reduction
  // one LDS array (a second __shared__ object can make hipcc drain the ring: §5 trap 4(a))
  //   [ring][rinv partials TPR x BM][row-sum partials 2 x BM][flag]
  __shared__ __attribute__((aligned(16))) unsigned char smem[RING + TPR * BM * 4 + 2 * BM * 4 + 16];
  const int mt = (a.M + BM - 1) / BM, nt = (a.N + BN - 1) / BN;
  const int bid = blockIdx.x;
  // Stream-K (SK, a.sk_table): a grid of about one workgroup per CU, each walking its host-built
  // list of (tile, k-step range) segments, so an output-tile count that is not a multiple of the CU
  // count (M = 320: 160 tiles of 64 x 64 for N = 2048) no longer idles the rest of the chip; a tile
  // split over several workgroups is combined by its last arriver from the write-through slabs in a
  // fixed order (ops.gemm.stream_k_table).  Otherwise exactly one (tile, split) unit per workgroup.
  if constexpr (!SK) {
    const int S = a.splits;
    // XCD-aware bijective remap (blocks b, b + 8, ... share an XCD -> contiguous logical ids)
    const int nwg = mt * nt * S, q8 = nwg >> 3, r8 = nwg & 7, xcd = bid & 7;
    const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int split = wgid % S, rest = wgid / S;
    const int kbeg = split * a.kchunk;
    int m_t = rest % mt, n_t = rest / mt;
    if (a.raster > 1 && mt > a.raster) {   // grouped raster (GemmArgs.raster)
      const int gsz = a.raster * nt, first = (rest / gsz) * a.raster;
      const int gm = min(mt - first, a.raster), in = rest % gsz;
      m_t = first + in % gm;
      n_t = in / gm;
    }
    tgemm_unit<BM, BN, EPI, STAGES, KS, NW, WK, NL, WGM, BKT, MF>(a, smem, a.M, S, S, split, m_t, n_t, kbeg,
                                                        max(0, (min(a.K, kbeg + a.kchunk) - kbeg) / KSTEP));
  } else {
    const int ng = gridDim.x, q8 = ng >> 3, r8 = ng & 7, xcd = bid & 7;
    const int wl = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    for (int sg = 0; sg < a.sk_segmax; ++sg) {
      const int4 e = *reinterpret_cast<const int4*>(a.sk_table + ((long)wl * a.sk_segmax + sg) * 4);
      if (e.x < 0) break;   // block-uniform: this workgroup's list ended
      tgemm_unit<BM, BN, EPI, STAGES, KS, NW, WK, NL, WGM, BKT, MF>(a, smem, a.M, e.w >> 16, a.sk_cmax, e.w & 0xffff, e.x % mt,
                                                          e.x / mt, e.y * KSTEP, e.z - e.y);
      __syncthreads();   // the next segment re-uses the ring, the row-scale partials and the flag
    }
  }
}

template <int BM, int BN, int EPI, int ST, int KS, int NW, int WK = 1, int NL = 0, int WGM = 2, bool SK = false,
          int BKT = 64, int MF = 16>
int launch_t(const GemmArgs& a, hipStream_t st) {
  const int mt = (a.M + BM - 1) / BM, nt = (a.N + BN - 1) / BN;
  const int grid = SK ? a.sk_grid : mt * nt * a.splits;
  hipLaunchKernelGGL((tgemm_kernel<BM, BN, EPI, ST, KS, NW, WK, NL, WGM, SK, BKT, MF>), dim3(grid),
                     dim3(64 * (NW * WK + NL)), 0, st, a);
  return (int)hipGetLastError();
}

// the stream-K instantiations: the one-split plans measured in stream-K mode, PLAIN epilogue only
// (they never beat the one-unit plans, profiles/r3_decode_gemm_panel.md section 5, so the autotuner
// does not offer them; tests/test_tgemm_gpu.py keeps the path honest); any other plan asked for in
// stream-K mode is refused (-25)
template <int BM, int BN, int EPI, int ST, int KS, int NW, int WK, int NL, int WGM>
constexpr bool sk_plan() {
  return EPI == EPI_PLAIN && WK == 1 &&
         ((BM == 64 && BN == 64 && ((NL == 0 && NW == 4 && ((ST == 3 && KS == 2) || (ST == 4 && KS == 1))) ||
                                    (NL == 4 && ST == 4) || (NL == 8 && ST == 4))) ||
          (BM == 64 && BN == 128 && NL == 0 && NW == 8 && ST == 3 && KS == 1) ||
          (BM == 128 && BN == 64 && NL == 4 && ST == 4));   // (160 x 128 spilled in the segment loop)
}

// Plans no measured shape ever selected: not instantiated, refused with -28.  The evidence is every
// autotune plan file of rounds 2-6 (42 files: TinyLlama, Llama-3-8B, Phi-3-mini, the MoE layers,
// decode buckets 1-512 and prefill buckets) plus ops.MOE_PLANS (profiles/r6_prune.md).
// ops.gemm._TG_PRUNED mirrors this
// table so the autotuner never proposes them.  Fields: BM, BN, stages, KS, compute waves, WK, NL,
// k depth, MFMA size.
struct PlanKey { int bm, bn, st, ks, nw, wk, nl, bkt, mf; };
constexpr PlanKey kPruned[] = {
    {64, 128, 6, 1, 4, 1, 0, 64, 16},  {64, 128, 2, 2, 4, 1, 0, 64, 16},  {128, 64, 3, 1, 4, 1, 0, 64, 16},
    {128, 64, 4, 1, 4, 1, 0, 64, 16},  {128, 64, 6, 1, 4, 1, 0, 64, 16},  {128, 64, 2, 2, 4, 1, 0, 64, 16},
    {128, 64, 3, 2, 4, 1, 0, 64, 16},  {128, 128, 3, 1, 4, 1, 0, 64, 16}, {128, 128, 4, 1, 4, 1, 0, 64, 16},
    {128, 128, 2, 2, 4, 1, 0, 64, 16}, {64, 128, 2, 1, 8, 1, 0, 64, 16},  {64, 128, 2, 2, 8, 1, 0, 64, 16},
    {128, 128, 2, 1, 8, 1, 0, 64, 16}, {128, 128, 2, 2, 8, 1, 0, 64, 16}, {192, 128, 2, 1, 8, 1, 0, 64, 16},
    {256, 128, 2, 1, 8, 1, 0, 64, 16}, {64, 128, 2, 2, 4, 2, 0, 64, 16},
    {128, 64, 2, 2, 4, 2, 0, 64, 16},  {128, 64, 3, 2, 4, 2, 0, 64, 16},  {128, 128, 2, 2, 4, 2, 0, 64, 16},
    {64, 64, 4, 1, 4, 1, 2, 64, 16},   {64, 64, 8, 1, 4, 1, 4, 64, 16},   {128, 128, 4, 1, 4, 1, 4, 64, 16},
    {256, 128, 6, 1, 8, 1, 0, 32, 16}, {256, 128, 6, 1, 8, 1, 8, 32, 16}, {128, 64, 4, 1, 4, 1, 8, 64, 32},
    {256, 128, 3, 1, 8, 1, 8, 64, 32}, {256, 256, 2, 1, 8, 1, 0, 64, 32},
};

template <int BM, int BN, int ST, int KS, int NW, int WK, int NL, int BKT, int MF>
constexpr bool pruned() {
  for (const PlanKey& p : kPruned)
    if (p.bm == BM && p.bn == BN && p.st == ST && p.ks == KS && p.nw == NW && p.wk == WK && p.nl == NL &&
        p.bkt == BKT && p.mf == MF)
      return true;
  return false;
}

template <int BM, int BN, int EPI, int ST, int KS, int NW, int WK = 1, int NL = 0, int WGM = 2, int BKT = 64, int MF = 16>
int launch_fit(const GemmArgs& a, hipStream_t st) {
  if constexpr (ST * KS * (BM + BN) * 2 * BKT > 150 * 1024) {
    return -9;  // ring does not fit the 160 KB LDS (with the epilogue scratch)
  } else if constexpr (pruned<BM, BN, ST, KS, NW, WK, NL, BKT, MF>()) {
    return -28;
  } else {
    if (a.sk_table != nullptr) {
      if constexpr (BKT == 64 && MF == 16 && sk_plan<BM, BN, EPI, ST, KS, NW, WK, NL, WGM>())
        return launch_t<BM, BN, EPI, ST, KS, NW, WK, NL, WGM, true>(a, st);
      else
        return -25;
    }
    return launch_t<BM, BN, EPI, ST, KS, NW, WK, NL, WGM, false, BKT, MF>(a, st);
  }
}

// 32 x 32 x 16 MFMA plans (GemmArgs.mfma = 32): the decode tiles the autotuner picks on the
// flagship (64 x 64 / 64 x 128 with k-step 128, the 128 x 64 and 256 x 128 loader-wave tiles) and
// the 256 x 256 prefill tile; chosen per shape by measurement like every other plan.  Only the
// 64-row forms are built (kPruned): the others lost 6-16 % to 16 x 16 x 32 (r6_gemm_fill_path.md)
template <int EPI>
int by_tile_m32(int bm, int bn, int stages, int ks, int nw, int nl, const GemmArgs& a, hipStream_t st) {
  if (nl == 0 && ks == 2 && stages == 3) {
    if (bm == 64 && bn == 64 && nw == 4) return launch_fit<64, 64, EPI, 3, 2, 4, 1, 0, 2, 64, 32>(a, st);
    if (bm == 64 && bn == 128 && nw == 8) return launch_fit<64, 128, EPI, 3, 2, 8, 1, 0, 2, 64, 32>(a, st);
  }
  if (nl == 0 && ks == 1 && bm == 256 && bn == 256 && nw == 8 && stages == 2)
    return launch_fit<256, 256, EPI, 2, 1, 8, 1, 0, 2, 64, 32>(a, st);
  if (nl == 8 && ks == 1 && bm == 128 && bn == 64 && nw == 4 && stages == 4)
    return launch_fit<128, 64, EPI, 4, 1, 4, 1, 8, 2, 64, 32>(a, st);
  if (nl == 8 && ks == 1 && bm == 256 && bn == 128 && nw == 8 && stages == 3)
    return launch_fit<256, 128, EPI, 3, 1, 8, 1, 8, 4, 64, 32>(a, st);
  return -27;
}

// 32-deep k-steps (GemmArgs.kdepth = 32): the 256-row tiles with 4-6 stage rings, for prefill-size
// M and the wide decode projections (gate/up), where a 64-deep ring of these tiles fits only 2-3
// stages in the 160 KB LDS.  256 x 256: 8 compute waves of 128 x 64 (2 x 4); 256 x 128: 64 x 64 (4 x 2)
template <int EPI>
int by_tile_k32(int bm, int bn, int stages, int nw, int nl, const GemmArgs& a, hipStream_t st) {
  // (256 x 256 with loader waves spills: 128 accumulators per lane leave no room at 3 waves/SIMD)
  if (bm == 256 && bn == 256 && nw == 8 && stages == 4 && nl == 0) return launch_fit<256, 256, EPI, 4, 1, 8, 1, 0, 2, 32>(a, st);
  if (bm == 256 && bn == 128 && nw == 8 && stages == 6) {
    if (nl == 0) return launch_fit<256, 128, EPI, 6, 1, 8, 1, 0, 4, 32>(a, st);
    if (nl == 8) return launch_fit<256, 128, EPI, 6, 1, 8, 1, 8, 4, 32>(a, st);
  }
  return -22;
}

// loader-wave tiles (NL > 0; KS 1): the decode-size plans the lab measured fastest
template <int EPI>
int by_tile_nl(int bm, int bn, int stages, int nw, int nl, const GemmArgs& a, hipStream_t st) {
  // batch <= 16: a 16-row tile (one 16 x 16 x 32 MFMA row block per wave, 4 waves across 128 columns,
  // WGM 1) streamed by 6 loader waves: the activation ring rows are 16, not 64 padded ones
  if (bm == 16 && bn == 128 && nw == 4 && nl == 6) {
    if (stages == 4) return launch_fit<16, 128, EPI, 4, 1, 4, 1, 6, 1>(a, st);
    if (stages == 8) return launch_fit<16, 128, EPI, 8, 1, 4, 1, 6, 1>(a, st);
  }
  if (bm == 64 && bn == 64 && nw == 4) {
    if (nl == 2 && stages == 4) return launch_fit<64, 64, EPI, 4, 1, 4, 1, 2>(a, st);
    if (nl == 4 && stages == 4) return launch_fit<64, 64, EPI, 4, 1, 4, 1, 4>(a, st);
    if (nl == 4 && stages == 8) return launch_fit<64, 64, EPI, 8, 1, 4, 1, 4>(a, st);
  }
  if (bm == 64 && bn == 64 && nw == 4 && nl == 8) {   // 8 loader waves: ~2x a 4-loader CU's intake
    if (stages == 4) return launch_fit<64, 64, EPI, 4, 1, 4, 1, 8>(a, st);
    if (stages == 8) return launch_fit<64, 64, EPI, 8, 1, 4, 1, 8>(a, st);
  }
  if (bm == 128 && bn == 64 && nw == 4 && stages == 4) {
    if (nl == 4) return launch_fit<128, 64, EPI, 4, 1, 4, 1, 4>(a, st);
    if (nl == 8) return launch_fit<128, 64, EPI, 4, 1, 4, 1, 8>(a, st);
  }
  if (bm == 128 && bn == 128 && nw == 4 && stages == 4) {
    if (nl == 4) return launch_fit<128, 128, EPI, 4, 1, 4, 1, 4>(a, st);
    if (nl == 8) return launch_fit<128, 128, EPI, 4, 1, 4, 1, 8>(a, st);
  }
  if (bm == 160 && bn == 128 && nw == 8 && stages == 3) {
    if (nl == 4) return launch_fit<160, 128, EPI, 3, 1, 8, 1, 4>(a, st);
    if (nl == 6) return launch_fit<160, 128, EPI, 3, 1, 8, 1, 6>(a, st);
  }
  if (bm == 256 && bn == 128 && nw == 8 && stages == 3) {   // 4 x 2 compute waves of 64 x 64
    if (nl == 4) return launch_fit<256, 128, EPI, 3, 1, 8, 1, 4, 4>(a, st);
    if (nl == 8) return launch_fit<256, 128, EPI, 3, 1, 8, 1, 8, 4>(a, st);
  }
  return -22;
}

template <int BM, int BN, int EPI, int NW>
int by_pipe(int stages, int ks, const GemmArgs& a, hipStream_t st) {
  if (ks == 1) return stages == 2 ? launch_fit<BM, BN, EPI, 2, 1, NW>(a, st) : launch_fit<BM, BN, EPI, 3, 1, NW>(a, st);
  return stages == 2 ? launch_fit<BM, BN, EPI, 2, 2, NW>(a, st) : launch_fit<BM, BN, EPI, 3, 2, NW>(a, st);
}

// deep rings (4 / 6 stages, k-step 64) for the 64- and 128-row tiles: at decode-size M a workgroup's
// k-loop is a chain of load latencies, so more stages = more bytes in flight per CU and a shorter
// chain (LDS holds up to 6 x 24 KB for 64 x 128; launch_fit rejects rings over 150 KB)
template <int BM, int BN, int EPI, int NW>
int by_pipe_deep(int stages, int ks, const GemmArgs& a, hipStream_t st) {
  if (ks == 1 && stages == 4) return launch_fit<BM, BN, EPI, 4, 1, NW>(a, st);
  if (ks == 1 && stages == 6) return launch_fit<BM, BN, EPI, 6, 1, NW>(a, st);
  return by_pipe<BM, BN, EPI, NW>(stages, ks, a, st);
}

// two k-groups of 4 waves (WK = 2, KS = 2; 2 or 3 stages) for the 4-wave tiles
template <int BM, int BN, int EPI>
int by_pipe_wk2(int stages, const GemmArgs& a, hipStream_t st) {
  return stages == 2 ? launch_fit<BM, BN, EPI, 2, 2, 4, 2>(a, st) : launch_fit<BM, BN, EPI, 3, 2, 4, 2>(a, st);
}

template <int EPI>
int by_tile(int bm, int bn, int stages, int ks, int nw, int wk, const GemmArgs& a, hipStream_t st) {
  if (wk == 2) {
    if (nw != 4 || ks != 2 || stages > 3) return -21;
    if (bm == 64 && bn == 64) return by_pipe_wk2<64, 64, EPI>(stages, a, st);
    if (bm == 64 && bn == 128) return by_pipe_wk2<64, 128, EPI>(stages, a, st);
    if (bm == 128 && bn == 64) return by_pipe_wk2<128, 64, EPI>(stages, a, st);
    if (bm == 128 && bn == 128) return by_pipe_wk2<128, 128, EPI>(stages, a, st);
    return -20;
  }
  if (nw == 4) {
    if (bm == 64 && bn == 64) return by_pipe_deep<64, 64, EPI, 4>(stages, ks, a, st);
    if (bm == 64 && bn == 128) return by_pipe_deep<64, 128, EPI, 4>(stages, ks, a, st);
    if (bm == 128 && bn == 64) return by_pipe_deep<128, 64, EPI, 4>(stages, ks, a, st);
    if (bm == 128 && bn == 128) return by_pipe_deep<128, 128, EPI, 4>(stages, ks, a, st);
  } else if (nw == 8) {
    if (bm == 64 && bn == 128) return by_pipe_deep<64, 128, EPI, 8>(stages, ks, a, st);
    if (bm == 128 && bn == 128) return by_pipe_deep<128, 128, EPI, 8>(stages, ks, a, st);
    if (bm == 192 && bn == 128) return by_pipe<192, 128, EPI, 8>(stages, ks, a, st);
    if (bm == 256 && bn == 128) return by_pipe<256, 128, EPI, 8>(stages, ks, a, st);
    if (bm == 256 && bn == 256) return by_pipe<256, 256, EPI, 8>(stages, ks, a, st);
  }
  return -20;
}

// Residual-stream helpers for the paths the GEMM epilogue cannot cover (first layer's embedding,
// tensor-parallel all-reduced outputs, MoE outputs): one wave per row, 16-B vectors.
//   res_add_ssq: r = bf16(h + r) in place (h may be null: r unchanged) and the row's partial sums
//   of squares, one per column slice of ``cw`` columns: ssq[slice * ssq_ld + m] (grid.y = slices,
//   so a decode-size M still spreads over many workgroups)
__global__ void __launch_bounds__(256) res_add_ssq_kernel(const u16* __restrict__ h, long ldh, u16* __restrict__ r,
                                                          long ldr, float* __restrict__ ssq, long ssq_ld, int M, int H,
                                                          int cw) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  u16* rr = r + (long)row * ldr;
  const u16* hr = h ? h + (long)row * ldh : nullptr;
  const int c1 = min(H, (int)(blockIdx.y + 1) * cw);
  float s = 0.f;
  for (int c = blockIdx.y * cw + lane * 8; c < c1; c += 512) {
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
  if (lane == 0) ssq[(long)blockIdx.y * ssq_ld + row] = s;
}

// ---- standalone epilogues for a vendor-GEMM output y (prefill-size M, where hipBLASLt's core is
// faster than tgemm's): the same math as EPI_QKV / EPI_SWIGLU applied to y = r . W'^T.
// lane-parallel: lane l sums slots l, l + 64, ... and the wave reduces (one load latency instead of
// a chain of n); every wave of the block computes it (no LDS, no barrier)
__device__ __forceinline__ float row_rinv(const float* ssq, int n, long ld, int m, float scale, float eps) {
  float s = 0.f;
  // 8 independent loads per lane per pass: a GEMV producer leaves hundreds of slots, which must
  // cost one round trip, not one per 64 slots
  for (int i0 = 0; i0 < n; i0 += 512) {
    float part[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 64 + (threadIdx.x & 63);
      part[u] = i < n ? ssq[(long)i * ld + m] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += part[u];
  }
  s = wave_sum(s);
  return rsqrtf(s * scale + eps);
}

// one block per row; a thread handles units of that row: 8 RoPE pairs (q/k: 16-B loads of both
// halves of a 32-column group, (c, c + 16)) or 8 V columns.  Units are numbered densely (no thread
// idles on the second half of a RoPE group) and one block covers the row: the previous layout (one
// block per (row, 2048-column slice), the owning thread of each half-group only) left half the
// q/k threads and most of the second slice idle and cost 8.9 us per call at the decode buckets
// (profiles/r6_end_kernels.md).  v_rows (decode, d = 64): V goes row-major to v_rows [M, nkv d],
// coalesced, and the decode attention kernel writes each sequence's newest V^T itself
// (gemm.qkv_rope_cache v_new), instead of 2-byte stores 32 B apart into the V^T cache.
__global__ void __launch_bounds__(256) qkv_post_kernel(const u16* __restrict__ y, long ldy, const float* __restrict__ ssq,
                                                       int ssq_n, long ssq_ld, float scale, float eps,
                                                       const int* __restrict__ pos, const float* __restrict__ cos_sin,
                                                       const int* __restrict__ slots, u16* __restrict__ q_out,
                                                       u16* __restrict__ kc, u16* __restrict__ vc, u16* __restrict__ v_rows,
                                                       int nq, int nkv, int d) {
  const int m = blockIdx.x;
  const float ri = ssq ? row_rinv(ssq, ssq_n, ssq_ld, m, scale, eps) : 1.f;
  const int hd = d / 2, qcols = nq * d, kcols = nkv * d, vcols = nkv * d;
  const int rope_units = (qcols + kcols) / 16, units = rope_units + vcols / 8;
  const int slot = slots[m];
  const long blk = slot >> 4, off = slot & 15;
  const float* cs = cos_sin + (long)pos[m] * d;
  const u16* yr = y + (long)m * ldy;
  for (int u = threadIdx.x; u < units; u += blockDim.x) {
    if (u < rope_units) {
      const int c = 32 * (u >> 1) + 8 * (u & 1);
      float x1[8], x2[8];
      unpack8(ld16(yr + c), x1);
      unpack8(ld16(yr + c + 16), x2);
      const bool isq = c < qcols;
      const int cc = isq ? c : c - qcols;
      const int head = cc / d, o = cc % d;
      const int d1 = 16 * (o >> 5) + (o & 15);
      float co[8], si[8];
      *(float4*)&co[0] = *(const float4*)(cs + d1);
      *(float4*)&co[4] = *(const float4*)(cs + d1 + 4);
      *(float4*)&si[0] = *(const float4*)(cs + hd + d1);
      *(float4*)&si[4] = *(const float4*)(cs + hd + d1 + 4);
      float r1[8], r2[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a1 = bfr(x1[j] * ri), a2 = bfr(x2[j] * ri);
        r1[j] = a1 * co[j] - a2 * si[j];
        r2[j] = a2 * co[j] + a1 * si[j];
      }
      u16* dst = isq ? q_out + ((long)m * nq + head) * d
                     : (slot >= 0 ? kc + ((blk * nkv + head) * 16 + off) * d : nullptr);
      if (dst) {
        st16(dst + d1, pack8(r1));
        st16(dst + hd + d1, pack8(r2));
      }
    } else {
      const int cc = 8 * (u - rope_units);
      float v[8];
      unpack8(ld16(yr + qcols + kcols + cc), v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] *= ri;
      if (v_rows) {
        st16(v_rows + (long)m * vcols + cc, pack8(v));
      } else if (slot >= 0) {
        const int head = cc / d, dim = cc % d;
        u16* vo = vc + ((blk * nkv + head) * d) * 16 + off;
#pragma unroll
        for (int j = 0; j < 8; ++j) vo[(long)(dim + j) * 16] = f2bf(v[j]);
      }
    }
  }
}

// act[m, 16 G + c] = silu(g) * u for the interleaved [g16 | u16] groups of y; one block per (row, 2048-output slice)
__global__ void __launch_bounds__(256) swiglu_post_kernel(const u16* __restrict__ y, long ldy, const float* __restrict__ ssq,
                                                          int ssq_n, long ssq_ld, float scale, float eps, u16* __restrict__ act,
                                                          long lda, int N) {
  const int m = blockIdx.x;
  const float ri = ssq ? row_rinv(ssq, ssq_n, ssq_ld, m, scale, eps) : 1.f;
  const u16* yr = y + (long)m * ldy;
  for (int o = (blockIdx.y * blockDim.x + threadIdx.x) * 8; o < N / 2; o += gridDim.y * blockDim.x * 8) {
    const int g = o >> 4, c = o & 15;
    float gv[8], uv[8];
    unpack8(ld16(yr + 32 * g + c), gv);
    unpack8(ld16(yr + 32 * g + 16 + c), uv);
#pragma unroll
    for (int j = 0; j < 8; ++j) gv[j] = silu(bfr(gv[j] * ri)) * bfr(uv[j] * ri);
    st16(act + (long)m * lda + o, pack8(gv));
  }
}
}  // namespace

extern "C" int dllm_qkv_post(const void* y, long ldy, const float* ssq, int ssq_n, long ssq_ld, float scale, float eps,
                             const int* pos, const float* cos_sin, const int* slots, void* q_out, void* kc, void* vc,
                             void* v_rows, int M, int nq, int nkv, int d, hipStream_t stream) {
  if (d % 32 || ldy % 8) return -1;
  if (M <= 0) return 0;
  const int units = (nq + nkv) * d / 16 + nkv * d / 8;
  const int threads = units <= 128 ? 128 : 256;
  hipLaunchKernelGGL(qkv_post_kernel, dim3(M), dim3(threads), 0, stream, (const u16*)y, ldy, ssq, ssq_n, ssq_ld, scale, eps,
                     pos, cos_sin, slots, (u16*)q_out, (u16*)kc, (u16*)vc, (u16*)v_rows, nq, nkv, d);
  return (int)hipGetLastError();
}

extern "C" int dllm_swiglu_post(const void* y, long ldy, const float* ssq, int ssq_n, long ssq_ld, float scale,
                                float eps, void* act, long lda, int M, int N, hipStream_t stream) {
  if (N % 32 || ldy % 8 || lda % 8) return -1;
  if (M <= 0) return 0;
  hipLaunchKernelGGL(swiglu_post_kernel, dim3(M, (N / 2 + 2047) / 2048), dim3(256), 0, stream, (const u16*)y, ldy, ssq, ssq_n, ssq_ld, scale,
                     eps, (u16*)act, lda, N);
  return (int)hipGetLastError();
}

// slices: column slices (ssq rows) to split H into; returns the slice count used (< 0: error)
extern "C" int dllm_res_add_ssq(const void* h, long ldh, void* r, long ldr, float* ssq, long ssq_ld, int slices, int M,
                                int H, hipStream_t stream) {
  if (H % 8 || ldr % 8 || (h && ldh % 8) || slices < 1) return -1;
  const int cw = ((H + slices - 1) / slices + 511) / 512 * 512;  // whole 512-column wave passes
  const int n = (H + cw - 1) / cw;
  if (M <= 0) return n;
  hipLaunchKernelGGL(res_add_ssq_kernel, dim3((M + 3) / 4, n), dim3(256), 0, stream, (const u16*)h, ldh, (u16*)r, ldr,
                     ssq, ssq_ld, M, H, cw);
  const int e = (int)hipGetLastError();
  return e ? -100 - e : n;
}

extern "C" int dllm_tgemm_sizeof_args() { return (int)sizeof(GemmArgs); }

// Host contract (checked again by csrc/bindings.cpp): K % 64 == 0, 16-B aligned rows (lda % 8),
// splits >= 1 with kchunk % 64 == 0, part >= splits * tiles * bm * bn floats and counters >= tiles
// (zeroed) when splits > 1; QKV/SWIGLU need N % 32 == 0 (and d % 32 == 0).
extern "C" int dllm_tgemm(const void* args, int bm, int bn, int stages, int ks, int nw, int wk, int epi,
                          hipStream_t stream, int nl) {
  const GemmArgs& a = *reinterpret_cast<const GemmArgs*>(args);
  if (a.M <= 0 || a.N <= 0) return 0;
  if (a.sk_table != nullptr && (!a.part || !a.counters || a.sk_grid < 1 || a.sk_segmax < 1 || a.sk_cmax < 1 ||
                                a.g_tiles != nullptr || a.splits != 1))
    return -24;
  if (a.mfma == 32) {     // 32 x 32 x 16 MFMA plans: one k-group, no MoE gather, no stream-K, k-step 64
    if (wk != 1 || a.g_tiles != nullptr || a.sk_table != nullptr || (a.kdepth != 0 && a.kdepth != 64) ||
        a.K % (BK * ks) || a.kchunk % (BK * ks) || a.kchunk <= 0 || a.splits < 1 || a.lda % 8 || a.N % 8 ||
        (a.Y && a.ldy % 8))
      return -23;
    if (a.splits > 1 && (!a.part || !a.counters)) return -2;
    if ((epi == EPI_QKV || epi == EPI_SWIGLU) && (a.N % 32)) return -3;
    if (epi == EPI_QKV && (a.d % 32 || !a.q_out || !a.kc || !a.vc || !a.pos || !a.slots || !a.cos_sin)) return -4;
    switch (epi) {
      case EPI_PLAIN: return by_tile_m32<EPI_PLAIN>(bm, bn, stages, ks, nw, nl, a, stream);
      case EPI_RESADD: return by_tile_m32<EPI_RESADD>(bm, bn, stages, ks, nw, nl, a, stream);
      case EPI_QKV: return by_tile_m32<EPI_QKV>(bm, bn, stages, ks, nw, nl, a, stream);
      case EPI_SWIGLU: return by_tile_m32<EPI_SWIGLU>(bm, bn, stages, ks, nw, nl, a, stream);
      case EPI_GELU: return by_tile_m32<EPI_GELU>(bm, bn, stages, ks, nw, nl, a, stream);
      default: return -6;
    }
  }
  if (a.mfma != 0 && a.mfma != 16) return -28;
  if (a.kdepth == 32) {   // 32-deep k-step plans: KS 1, one k-group, no MoE gather, no stream-K
    if (ks != 1 || wk != 1 || a.g_tiles != nullptr || a.sk_table != nullptr || a.K % BK || a.kchunk % BK ||
        a.kchunk <= 0 || a.splits < 1 || a.lda % 8 || a.N % 8 || (a.Y && a.ldy % 8))
      return -23;
    if (a.splits > 1 && (!a.part || !a.counters)) return -2;
    if ((epi == EPI_QKV || epi == EPI_SWIGLU) && (a.N % 32)) return -3;
    if (epi == EPI_QKV && (a.d % 32 || !a.q_out || !a.kc || !a.vc || !a.pos || !a.slots || !a.cos_sin)) return -4;
    switch (epi) {
      case EPI_PLAIN: return by_tile_k32<EPI_PLAIN>(bm, bn, stages, nw, nl, a, stream);
      case EPI_RESADD: return by_tile_k32<EPI_RESADD>(bm, bn, stages, nw, nl, a, stream);
      case EPI_QKV: return by_tile_k32<EPI_QKV>(bm, bn, stages, nw, nl, a, stream);
      case EPI_SWIGLU: return by_tile_k32<EPI_SWIGLU>(bm, bn, stages, nw, nl, a, stream);
      case EPI_GELU: return by_tile_k32<EPI_GELU>(bm, bn, stages, nw, nl, a, stream);
      default: return -6;
    }
  }
  if (a.kdepth != 0 && a.kdepth != 64) return -26;
  if (nl > 0) {   // loader-wave plans: KS 1, one k-group, no MoE gather
    if (ks != 1 || wk != 1 || a.g_tiles != nullptr || a.K % BK || a.kchunk % BK || a.kchunk <= 0 || a.splits < 1 ||
        a.lda % 8 || a.N % 8 || (a.Y && a.ldy % 8))
      return -23;
    if (a.splits > 1 && (!a.part || !a.counters)) return -2;
    if ((epi == EPI_QKV || epi == EPI_SWIGLU) && (a.N % 32)) return -3;
    if (epi == EPI_QKV && (a.d % 32 || !a.q_out || !a.kc || !a.vc || !a.pos || !a.slots || !a.cos_sin)) return -4;
    switch (epi) {
      case EPI_PLAIN: return by_tile_nl<EPI_PLAIN>(bm, bn, stages, nw, nl, a, stream);
      case EPI_RESADD: return by_tile_nl<EPI_RESADD>(bm, bn, stages, nw, nl, a, stream);
      case EPI_QKV: return by_tile_nl<EPI_QKV>(bm, bn, stages, nw, nl, a, stream);
      case EPI_SWIGLU: return by_tile_nl<EPI_SWIGLU>(bm, bn, stages, nw, nl, a, stream);
      case EPI_GELU: return by_tile_nl<EPI_GELU>(bm, bn, stages, nw, nl, a, stream);
      default: return -6;
    }
  }
  if ((ks != 1 && ks != 2) || (nw != 4 && nw != 8) || (wk != 1 && wk != 2)) return -8;
  if (a.K % (BK * ks) || a.kchunk % (BK * ks) || a.kchunk <= 0 || a.splits < 1 || a.lda % 8) return -1;
  if (a.splits > 1 && (!a.part || !a.counters)) return -2;
  if ((epi == EPI_QKV || epi == EPI_SWIGLU) && (a.N % 32)) return -3;
  if (a.N % 8 || (a.Y && a.ldy % 8)) return -7;  // 16-B output row vectors
  if (epi == EPI_QKV && (a.d % 32 || !a.q_out || !a.kc || !a.vc || !a.pos || !a.slots || !a.cos_sin)) return -4;
  if (a.g_tiles != nullptr && (a.splits != 1 || a.M != a.g_max * bm || epi == EPI_QKV || a.ssq_in || a.w_panel))
    return -10;
  if (stages < 2 || stages > 6 || stages == 5 || (stages > 3 && (ks != 1 || bm > 128))) return -5;
  switch (epi) {
    case EPI_PLAIN: return by_tile<EPI_PLAIN>(bm, bn, stages, ks, nw, wk, a, stream);
    case EPI_RESADD: return by_tile<EPI_RESADD>(bm, bn, stages, ks, nw, wk, a, stream);
    case EPI_QKV: return by_tile<EPI_QKV>(bm, bn, stages, ks, nw, wk, a, stream);
    case EPI_SWIGLU: return by_tile<EPI_SWIGLU>(bm, bn, stages, ks, nw, wk, a, stream);
    case EPI_GELU: return by_tile<EPI_GELU>(bm, bn, stages, ks, nw, wk, a, stream);
    default: return -6;
  }
}
