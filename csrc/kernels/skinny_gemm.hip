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
