// Decode-shaped GEMM  Y[M, N] = X[M, K] . W[N, K]^T  (+ optional fused SwiGLU on the X load),
// M <= 128, bf16 in / f32 accumulate / bf16 out, on mfma_f32_16x16x32_bf16.
//
// Why: at decode batch sizes the weight matrix is streamed exactly once and the work is
// HBM-bound; hipBLASLt's kernels for these shapes sit at an ~18 us floor (0.45-2.5 TB/s on
// 8-46 MB weights, measured on MI355X).  Here:
//   * every wave owns NTW 16-column tiles x MT 16-row tiles and a contiguous K range; weight
//     fragments are one 16-B load per lane straight to VGPRs (the 'GEMV / M <= 16' row of the
//     guide's staging table: no LDS round trip for an operand that is read once), issued UNROLL
//     k-steps ahead;
//   * X (activations, <= 128 x K, L2-resident and re-read by every workgroup) is also loaded
//     per fragment from L2;
//   * the 4 waves of a workgroup split K 4 ways and are reduced through LDS;
//   * grid.y splits K across workgroups (split-K) so that even N = 2048 yields >= 256
//     workgroups; the split partials are combined IN the kernel by the last-arriving workgroup
//     of each column tile (agent-scope release/acquire ticket: cdna_hip_programming.md §5
//     'In-launch split-K reduction', Guideline 16) -> one launch, graph-capturable, counters
//     reset by the reducer;
//   * SWIGLU=true: X is the fused gate|up GEMM output [M, 2K] and the kernel computes
//     silu(gate) * up on the fly while loading X (the down projection absorbs the activation).
// Tile / split choice per (M, N, K) is autotuned on the host (ops.gemm).
#include "common.h"

namespace {

template <int MT, int NTW, bool SWIGLU>
__global__ void __launch_bounds__(256) skinny_gemm_kernel(const u16* __restrict__ X, long ldx,
                                                          const u16* __restrict__ W, u16* __restrict__ Y, long ldy,
                                                          int M, int N, int K, int kchunk, float* __restrict__ part,
                                                          int* __restrict__ counters) {
  constexpr int NC = 16 * NTW;  // columns per workgroup
  __shared__ float s_red[2][MT * 16][NC + 1];
  __shared__ int s_last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int tile = blockIdx.x, split = blockIdx.y, S = gridDim.y;
  const int col0 = tile * NC;
  const int kbeg = split * kchunk;
  const int kend = min(K, kbeg + kchunk);
  // contiguous K range of this wave (multiple of 32)
  const int klen = kend - kbeg;
  int kw = (((klen + 3) / 4) + 31) & ~31;
  const int wk0 = kbeg + wave * kw;
  const int wk1 = min(kend, wk0 + kw);

  f32x4 acc[MT][NTW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const u16* wrow[NTW];
#pragma unroll
  for (int n = 0; n < NTW; ++n) {
    int c = col0 + 16 * n + r16;
    c = c < N ? c : N - 1;  // clamp (results for c >= N are discarded)
    wrow[n] = W + (long)c * K + 8 * g;
  }
  const u16* xrow[MT];
  bool xok[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int r = 16 * m + r16;
    xok[m] = r < M;
    xrow[m] = X + (long)(xok[m] ? r : 0) * ldx + 8 * g;
  }

  // Software pipeline: the loads of block i+1 (U k-steps of W and X) are in flight while the
  // MFMAs of block i run (two register stages, ping-pong, fully unrolled -> static indexing).
  constexpr int U = MT >= 8 ? 1 : (MT >= 4 ? 2 : 4);
  struct Stage {
    bf16x8 w[U][NTW];
    uint4 x[U][MT];
    uint4 xu[SWIGLU ? U : 1][SWIGLU ? MT : 1];
  };
  auto load = [&](Stage& st, int k0) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int n = 0; n < NTW; ++n) st.w[u][n] = ldnt_bf16x8(wrow[n] + k0 + 32 * u);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        st.x[u][m] = ld16(xrow[m] + k0 + 32 * u);
        if constexpr (SWIGLU) st.xu[u][m] = ld16(xrow[m] + K + k0 + 32 * u);
      }
  };
  auto compute = [&](const Stage& st) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bf16x8 xf[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        uint4 v = st.x[u][m];
        if constexpr (SWIGLU) {
          float gt[8], up[8];
          unpack8(v, gt);
          unpack8(st.xu[u][m], up);
#pragma unroll
          for (int j = 0; j < 8; ++j) gt[j] = gt[j] / (1.f + __expf(-gt[j])) * up[j];
          v = pack8(gt);
        }
        if (!xok[m]) v = make_uint4(0, 0, 0, 0);
        xf[m] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NTW; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[m], st.w[u][n], acc[m][n], 0, 0, 0);
    }
  };
  const int nblk = (wk1 > wk0) ? (wk1 - wk0) / (32 * U) : 0;
  int kb = wk0;
  if (nblk > 0) {
    Stage A, B;
    load(A, kb);
    for (int i = 0; i < nblk; i += 2) {
      if (i + 1 < nblk) load(B, kb + 32 * U);
      compute(A);
      if (i + 1 < nblk) {
        if (i + 2 < nblk) load(A, kb + 64 * U);
        compute(B);
      }
      kb += 64 * U;
    }
    kb = wk0 + nblk * 32 * U;
  }
  for (; kb < wk1; kb += 32) {  // tail (< U k-steps)
    Stage T;
#pragma unroll
    for (int n = 0; n < NTW; ++n) T.w[0][n] = ldnt_bf16x8(wrow[n] + kb);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      T.x[0][m] = ld16(xrow[m] + kb);
      if constexpr (SWIGLU) T.xu[0][m] = ld16(xrow[m] + K + kb);
    }
    // compute only u = 0
    bf16x8 xf[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      uint4 v = T.x[0][m];
      if constexpr (SWIGLU) {
        float gt[8], up[8];
        unpack8(v, gt);
        unpack8(T.xu[0][m], up);
#pragma unroll
        for (int j = 0; j < 8; ++j) gt[j] = gt[j] / (1.f + __expf(-gt[j])) * up[j];
        v = pack8(gt);
      }
      if (!xok[m]) v = make_uint4(0, 0, 0, 0);
      xf[m] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NTW; ++n)
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[m], T.w[0][n], acc[m][n], 0, 0, 0);
  }

  // ---- reduce the 4 waves in a fixed order ((w0 + w2) + (w1 + w3)): bitwise reproducible.
  // C layout: acc[m][n][r] = C[row 16m + 4g + r][col 16n + r16]
#define DLLM_FOR_C(BODY)                                                          \
  _Pragma("unroll") for (int m = 0; m < MT; ++m)                                  \
  _Pragma("unroll") for (int n = 0; n < NTW; ++n)                                 \
  _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                 \
    float& slot_ = s_red[SLOT][16 * m + 4 * g + r][16 * n + r16];                 \
    BODY;                                                                         \
  }
  if (wave >= 2) {
    const int SLOT = wave - 2;
    DLLM_FOR_C(slot_ = acc[m][n][r])
  }
  __syncthreads();
  if (wave < 2) {
    const int SLOT = wave;
    DLLM_FOR_C(acc[m][n][r] += slot_)
  }
  __syncthreads();
  if (wave == 1) {
    const int SLOT = 0;
    DLLM_FOR_C(slot_ = acc[m][n][r])
  }
  __syncthreads();
  if (wave == 0) {
    const int SLOT = 1;
    DLLM_FOR_C(slot_ = acc[m][n][r] + s_red[0][16 * m + 4 * g + r][16 * n + r16])
  }
#undef DLLM_FOR_C
  __syncthreads();
  const int rows = min(M, MT * 16);
  if (S == 1) {
    for (int e = threadIdx.x; e < rows * NC; e += 256) {
      const int row = e / NC, c = e % NC;
      if (col0 + c < N) Y[(long)row * ldy + col0 + c] = f2bf(s_red[1][row][c]);
    }
    return;
  }
  // ---- split-K: write-through slab store, ticket; the last arriver reduces (sc1 loads)
  const long slab_elems = (long)(MT * 16) * NC;
  const __amdgpu_buffer_rsrc_t pr = make_rsrc(part, (unsigned)min((long)gridDim.x * gridDim.y * slab_elems * 4, 0x7fffffffL));
  const unsigned my_off = (unsigned)(((long)split * gridDim.x + tile) * slab_elems * 4);
  for (int e = threadIdx.x * 4; e < rows * NC; e += 1024) {
    const int row = e / NC, c = e % NC;
    st_wt16(pr, my_off + e * 4, make_float4(s_red[1][row][c], s_red[1][row][c + 1], s_red[1][row][c + 2], s_red[1][row][c + 3]));
  }
  if (!ticket_last(&counters[tile], S, &s_last)) return;
  for (int e = threadIdx.x * 4; e < rows * NC; e += 1024) {
    const int row = e / NC, c = e % NC;
    float4 v = {0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < S; ++sp) {
      const float4 q = ld_wt16(pr, (unsigned)((((long)sp * gridDim.x + tile) * slab_elems + e) * 4));
      v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
    }
    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (col0 + c + j < N) Y[(long)row * ldy + col0 + c + j] = f2bf(vv[j]);
  }
}

// ---- small-batch decode GEMM with the fused decoder epilogues (M <= 16; ops.gemm "skinnyE" core)
//
// At batch 2-8 a decode projection is a weight stream, but the plain kernel above could not carry
// the decoder layer's epilogues, so the autotuner paired it with a standalone epilogue launch (5-7 us
// at M = 8, as much as the GEMM) or fell back to an LDS-tiled tgemm plan (10-15 us; the fused GEMV
// is VALU-bound at 8 rows: 8.5 VALU ops per weight byte).  This kernel keeps the MFMA fragments
// (one 16-B weight load per lane straight to VGPRs, 4 k-steps in flight per stage, two stages) and:
//   * PANEL: reads the K-panel-major weight copy the fused tgemm plans stream ([K/64][N][64], the
//     model keeps it): a 16-row fragment pair of one panel is 2 KB contiguous (16 rows x 128 B) instead
//     of 16 pieces of 64 B K x 2 bytes apart;
//   * EPI: the 4 waves' partial tiles (and split-K partials, combined by the tile's last arriver)
//     end in one LDS tile [16 rows][NC], from which the epilogue runs: residual add + per-tile row
//     sums of squares (RESADD), folded RMSNorm row scale + RoPE + q / paged K / V^T writes (QKV),
//     folded RMSNorm + silu(g) * u (SWIGLU) - the same math and roundings as tgemm's epilogues.
//     QKV / SWIGLU need NTW = 2: a workgroup owns a whole 32-column group, so every (c, c + 16)
//     pair of the permuted q/k rows and of the interleaved gate/up rows is in its tile.
struct SkEpi {
  u16* res;           // RESADD: residual [M, ldr], updated in place
  long ldr;
  float* ssq_out;     // RESADD: per-tile partial row sums of r^2: ssq_out[tile * ssq_out_ld + m]
  long ssq_out_ld;
  const float* ssq_in;  // QKV / SWIGLU: producer partials [ssq_n][ssq_in_ld]
  int ssq_n;
  long ssq_in_ld;
  float scale, eps;
  const int* pos;
  const float* cos_sin;
  const int* slots;
  u16* q_out;
  u16* kc;
  u16* vc;
  int nq, nkv, d;
};
enum { SK_PLAIN = 0, SK_RESADD = 1, SK_QKV = 2, SK_SWIGLU = 3 };

template <int NTW, bool PANEL, int EPI>
__global__ void __launch_bounds__(256) skinny_epi_kernel(const u16* __restrict__ X, long ldx,
                                                         const u16* __restrict__ W, u16* __restrict__ Y, long ldy,
                                                         int M, int N, int K, int kchunk, float* __restrict__ part,
                                                         int* __restrict__ counters, SkEpi ea) {
  static_assert(EPI == SK_PLAIN || EPI == SK_RESADD || NTW == 2, "paired epilogues need 32-column tiles");
  constexpr int NC = 16 * NTW;
  __shared__ float s_red[2][16][NC + 1];
  __shared__ float s_ri[16];
  __shared__ int s_last;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int tile = blockIdx.x, split = blockIdx.y, S = gridDim.y;
  const int col0 = tile * NC;
  const int kbeg = split * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int klen = kend - kbeg;
  const int kw = (((klen + 3) / 4) + 31) & ~31;
  const int wk0 = kbeg + wave * kw;
  const int wk1 = min(kend, wk0 + kw);

  f32x4 acc[NTW];
#pragma unroll
  for (int n = 0; n < NTW; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const u16* wb[NTW];
#pragma unroll
  for (int n = 0; n < NTW; ++n) {
    const int c = min(col0 + 16 * n + r16, N - 1);
    wb[n] = PANEL ? W + (long)c * 64 + 8 * g : W + (long)c * K + 8 * g;
  }
  auto wptr = [&](int n, int k) -> const u16* {
    return PANEL ? wb[n] + (long)(k >> 6) * N * 64 + (k & 63) : wb[n] + k;
  };
  const bool xok = r16 < M;
  const u16* xrow = X + (long)(xok ? r16 : 0) * ldx + 8 * g;

  constexpr int U = 4;
  struct Stage {
    bf16x8 w[U][NTW];
    uint4 x[U];
  };
  auto load = [&](Stage& st, int k0) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int n = 0; n < NTW; ++n) st.w[u][n] = ldnt_bf16x8(wptr(n, k0 + 32 * u));
#pragma unroll
    for (int u = 0; u < U; ++u) st.x[u] = ld16(xrow + k0 + 32 * u);
  };
  auto compute = [&](const Stage& st, int uu) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= uu) break;
      const bf16x8 xf = __builtin_bit_cast(bf16x8, xok ? st.x[u] : make_uint4(0, 0, 0, 0));
#pragma unroll
      for (int n = 0; n < NTW; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf, st.w[u][n], acc[n], 0, 0, 0);
    }
  };
  // folded RMSNorm row scale (QKV / SWIGLU): the producer's partial sums, summed lane-parallel while
  // the first weight stage is in flight
  const int nblk = (wk1 > wk0) ? (wk1 - wk0) / (32 * U) : 0;
  Stage A, B;
  if (nblk > 0) load(A, wk0);
  if constexpr (EPI == SK_QKV || EPI == SK_SWIGLU) {
    for (int m = wave; m < M; m += 4) {
      float sacc = 0.f;
      for (int i0 = 0; i0 < ea.ssq_n; i0 += 512) {
        float pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u * 64 + lane;
          pp[u] = i < ea.ssq_n ? ea.ssq_in[(long)i * ea.ssq_in_ld + m] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) sacc += pp[u];
      }
      sacc = wave_sum(sacc);
      if (lane == 0) s_ri[m] = rsqrtf(sacc * ea.scale + ea.eps);
    }
  }
  int kb = wk0;
  for (int i = 0; i < nblk; i += 2) {
    if (i + 1 < nblk) load(B, kb + 32 * U);
    compute(A, U);
    if (i + 1 < nblk) {
      if (i + 2 < nblk) load(A, kb + 64 * U);
      compute(B, U);
    }
    kb += 64 * U;
  }
  kb = wk0 + nblk * 32 * U;
  if (kb < wk1) {  // tail: fewer than U k-steps
    Stage T;
    const int tail = (wk1 - kb) / 32;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= tail) break;
#pragma unroll
      for (int n = 0; n < NTW; ++n) T.w[u][n] = ldnt_bf16x8(wptr(n, kb + 32 * u));
      T.x[u] = ld16(xrow + kb + 32 * u);
    }
    compute(T, tail);
  }

  // ---- reduce the 4 waves in a fixed order ((w0 + w2) + (w1 + w3)) into s_red[1]
  // C layout: acc[n][r] = C[row 4g + r][col 16n + r16]
#define DLLM_SK_FOR_C(BODY)                                 \
  _Pragma("unroll") for (int n = 0; n < NTW; ++n)           \
  _Pragma("unroll") for (int r = 0; r < 4; ++r) {           \
    float& slot_ = s_red[SLOT][4 * g + r][16 * n + r16];    \
    BODY;                                                   \
  }
  if (wave >= 2) { const int SLOT = wave - 2; DLLM_SK_FOR_C(slot_ = acc[n][r]) }
  __syncthreads();
  if (wave < 2) { const int SLOT = wave; DLLM_SK_FOR_C(acc[n][r] += slot_) }
  __syncthreads();
  if (wave == 1) { const int SLOT = 0; DLLM_SK_FOR_C(slot_ = acc[n][r]) }
  __syncthreads();
  if (wave == 0) { const int SLOT = 1; DLLM_SK_FOR_C(slot_ = acc[n][r] + s_red[0][4 * g + r][16 * n + r16]) }
#undef DLLM_SK_FOR_C
  __syncthreads();
  const int rows = min(M, 16);
  if (S > 1) {  // write-through slabs, ticket; the last arriver sums them back into s_red[1]
    constexpr long slab = 16L * NC;
    const __amdgpu_buffer_rsrc_t pr = make_rsrc(part, (unsigned)min((long)gridDim.x * gridDim.y * slab * 4, 0x7fffffffL));
    const unsigned my_off = (unsigned)(((long)split * gridDim.x + tile) * slab * 4);
    for (int e = threadIdx.x * 4; e < rows * NC; e += 1024) {
      const int row = e / NC, c = e % NC;
      st_wt16(pr, my_off + e * 4, make_float4(s_red[1][row][c], s_red[1][row][c + 1], s_red[1][row][c + 2], s_red[1][row][c + 3]));
    }
    if (!ticket_last(&counters[tile], S, &s_last)) return;
    for (int e = threadIdx.x * 4; e < rows * NC; e += 1024) {
      const int row = e / NC, c = e % NC;
      float4 v = {0.f, 0.f, 0.f, 0.f};
      for (int sp = 0; sp < S; ++sp) {
        const float4 q = ld_wt16(pr, (unsigned)((((long)sp * gridDim.x + tile) * slab + e) * 4));
        v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
      }
      s_red[1][row][c] = v.x; s_red[1][row][c + 1] = v.y; s_red[1][row][c + 2] = v.z; s_red[1][row][c + 3] = v.w;
    }
    __syncthreads();
  }

  // ---- epilogue from the LDS tile
  if constexpr (EPI == SK_PLAIN) {
    for (int e = threadIdx.x; e < rows * NC; e += 256) {
      const int row = e / NC, c = e % NC;
      if (col0 + c < N) Y[(long)row * ldy + col0 + c] = f2bf(s_red[1][row][c]);
    }
  } else if constexpr (EPI == SK_RESADD) {
    // r = bf16(bf16(acc) + r) (res_add_ssq numerics); s_red[0] collects r^2 for the tile's row sums
    for (int e = threadIdx.x; e < rows * NC; e += 256) {
      const int row = e / NC, c = e % NC;
      float v2 = 0.f;
      if (col0 + c < N) {
        u16* p = ea.res + (long)row * ea.ldr + col0 + c;
        const float v = bf2f(f2bf(bf2f(f2bf(s_red[1][row][c])) + bf2f(*p)));
        *p = f2bf(v);
        v2 = v * v;
      }
      s_red[0][row][c] = v2;
    }
    __syncthreads();
    if (threadIdx.x < rows) {
      float ss = 0.f;
      for (int c = 0; c < NC; ++c) ss += s_red[0][threadIdx.x][c];   // fixed order: reproducible
      ea.ssq_out[(long)tile * ea.ssq_out_ld + threadIdx.x] = ss;
    }
  } else {
    // (c, c + 16) pairs of the 32-column group col0: thread -> (row, pair)
    for (int e = threadIdx.x; e < rows * 16; e += 256) {
      const int m = e / 16, p = e % 16;
      const float ri = s_ri[m];
      const float x1 = s_red[1][m][p], x2 = s_red[1][m][p + 16];
      if constexpr (EPI == SK_SWIGLU) {
        const float gv = bf2f(f2bf(x1 * ri)), uv = bf2f(f2bf(x2 * ri));
        Y[(long)m * ldy + col0 / 2 + p] = f2bf(gv / (1.f + __expf(-gv)) * uv);
      } else {
        const int d = ea.d, hd = d / 2, qcols = ea.nq * d, kcols = ea.nkv * d;
        const int c = col0 + p, slot = ea.slots[m];
        const long blk = slot >> 4, off = slot & 15;
        if (c < qcols + kcols) {
          const bool isq = c < qcols;
          const int cc = isq ? c : c - qcols, head = cc / d, o = cc % d;
          const int d1 = 16 * (o >> 5) + (o & 15);
          const float* cs = ea.cos_sin + (long)ea.pos[m] * d;
          const float a1 = bf2f(f2bf(x1 * ri)), a2 = bf2f(f2bf(x2 * ri));
          const float co = cs[d1], si = cs[hd + d1];
          u16* dst = isq ? ea.q_out + ((long)m * ea.nq + head) * d
                         : (slot >= 0 ? ea.kc + ((blk * ea.nkv + head) * 16 + off) * d : nullptr);
          if (dst) {
            dst[d1] = f2bf(a1 * co - a2 * si);
            dst[hd + d1] = f2bf(a2 * co + a1 * si);
          }
        } else if (slot >= 0) {
          const int cc = c - qcols - kcols, head = cc / d, dim = cc % d;  // V columns: unpermuted
          u16* vo = ea.vc + ((blk * ea.nkv + head) * d) * 16 + off;
          vo[(long)dim * 16] = f2bf(x1 * ri);
          vo[(long)(dim + 16) * 16] = f2bf(x2 * ri);
        }
      }
    }
  }
}

template <int NTW, bool PANEL, int EPI>
int launch_epi(const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K, int splits, float* part,
               int* counters, const SkEpi& ea, hipStream_t st) {
  const int tiles = (N + 16 * NTW - 1) / (16 * NTW);
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + 31) & ~31;
  const int S = (K + kchunk - 1) / kchunk;
  hipLaunchKernelGGL((skinny_epi_kernel<NTW, PANEL, EPI>), dim3(tiles, S), dim3(256), 0, st, (const u16*)X, ldx,
                     (const u16*)W, (u16*)Y, ldy, M, N, K, kchunk, part, counters, ea);
  return (int)hipGetLastError();
}

template <bool PANEL>
int epi_by(int ntw, int epi, const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K, int splits,
           float* part, int* counters, const SkEpi& ea, hipStream_t st) {
  switch (epi) {
    case SK_PLAIN:
      return ntw == 1 ? launch_epi<1, PANEL, SK_PLAIN>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, ea, st)
                      : launch_epi<2, PANEL, SK_PLAIN>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, ea, st);
    case SK_RESADD:
      return ntw == 1 ? launch_epi<1, PANEL, SK_RESADD>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, ea, st)
                      : launch_epi<2, PANEL, SK_RESADD>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, ea, st);
    case SK_QKV: return launch_epi<2, PANEL, SK_QKV>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, ea, st);
    case SK_SWIGLU: return launch_epi<2, PANEL, SK_SWIGLU>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, ea, st);
    default: return -7;
  }
}

template <int MT, int NTW, bool SW>
int launch(const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K, int splits, float* part,
           int* counters, hipStream_t st) {
  const int tiles = (N + 16 * NTW - 1) / (16 * NTW);
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + 31) & ~31;
  const int S = (K + kchunk - 1) / kchunk;
  hipLaunchKernelGGL((skinny_gemm_kernel<MT, NTW, SW>), dim3(tiles, S), dim3(256), 0, st, (const u16*)X, ldx,
                     (const u16*)W, (u16*)Y, ldy, M, N, K, kchunk, part, counters);
  return (int)hipGetLastError();
}

template <int MT, bool SW>
int by_ntw(int ntw, const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K, int splits,
           float* part, int* counters, hipStream_t st) {
  switch (ntw) {
    case 1: return launch<MT, 1, SW>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
    case 2: return launch<MT, 2, SW>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
    case 4: return launch<MT, 4, SW>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
    default: return -10;
  }
}

template <bool SW>
int by_mt(int M, int ntw, const void* X, long ldx, const void* W, void* Y, long ldy, int N, int K, int splits,
          float* part, int* counters, hipStream_t st) {
  if (M <= 16) return by_ntw<1, SW>(ntw, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  if (M <= 32) return by_ntw<2, SW>(ntw, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  if (M <= 64) return by_ntw<4, SW>(ntw, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  if (M <= 128 && ntw <= 2) return by_ntw<8, SW>(ntw, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  return -11;
}
}  // namespace

// part: >= splits * ceil(N / (16 ntw)) * 16 * ceil(M/16) * 16 * ntw floats; counters: >= ceil(N/(16 ntw)) ints, zeroed.
extern "C" int dllm_skinny_gemm(const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K, int ntw,
                                int splits, int swiglu, float* part, int* counters, hipStream_t stream) {
  if (K % 32 != 0 || M <= 0 || M > 128 || splits < 1) return -1;
  if (splits > 1 && (!part || !counters)) return -2;
  return swiglu ? by_mt<true>(M, ntw, X, ldx, W, Y, ldy, N, K, splits, part, counters, stream)
                : by_mt<false>(M, ntw, X, ldx, W, Y, ldy, N, K, splits, part, counters, stream);
}

// Small-batch MFMA GEMM with a fused decoder epilogue (skinny_epi_kernel): M <= 16, K % 64 == 0
// (panel weights) or % 32, ntw 1 or 2 (2 for QKV / SWIGLU, which also need N % 32 == 0).  panel:
// W is the [K/64][N][64] copy.  RESADD writes ceil(N / (16 ntw)) row-sum slots.
extern "C" int dllm_skinny_epi(const void* X, long ldx, const void* W, int panel, void* Y, long ldy, int M, int N, int K,
                               int ntw, int splits, int epi, float* part, int* counters, void* res, long ldr,
                               float* ssq_out, long ssq_out_ld, const float* ssq_in, int ssq_n, long ssq_in_ld,
                               float scale, float eps, const int* pos, const float* cos_sin, const int* slots,
                               void* q_out, void* kc, void* vc, int nq, int nkv, int d, hipStream_t stream) {
  if (M <= 0 || M > 16 || K % (panel ? 64 : 32) || splits < 1 || (ntw != 1 && ntw != 2)) return -1;
  if (splits > 1 && (!part || !counters)) return -2;
  if ((epi == SK_QKV || epi == SK_SWIGLU) && (ntw != 2 || N % 32 || !ssq_in || ssq_n < 1)) return -3;
  if (epi == SK_QKV && (d % 32 || N != (nq + 2 * nkv) * d || !q_out || !kc || !vc || !pos || !cos_sin || !slots))
    return -4;
  if (epi == SK_RESADD && (!res || !ssq_out)) return -5;
  const SkEpi ea{(u16*)res, ldr, ssq_out, ssq_out_ld, ssq_in, ssq_n, ssq_in_ld, scale, eps, pos, cos_sin, slots,
                 (u16*)q_out, (u16*)kc, (u16*)vc, nq, nkv, d};
  return panel ? epi_by<true>(ntw, epi, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, ea, stream)
               : epi_by<false>(ntw, epi, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, ea, stream);
}
