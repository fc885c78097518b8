// Decode GEMM for mid-size batches, 64 < M <= 256:  Y[M, N] = X[M, K] . W[N, K]^T  (+ fused SwiGLU).
//
// Why: at M = 128-256 the step's weights (the whole model, every decode step) are still streamed
// once from HBM, but hipBLASLt sits at 0.7-2.5 TB/s on these shapes (10-27 us per GEMM measured:
// scripts/gemm_probe.py, profiles/).  Layout of one workgroup (4 waves, 256 threads):
//   * tile = ALL rows (BM = 64 MT, waves stacked along M: wave w owns rows [16 MT w, 16 MT (w+1)))
//     x BN = 16 NT columns, so every weight byte is read from HBM exactly once per split;
//   * the W tile [BN x 64 k] is staged in LDS (double-buffered, one barrier per 64-k block) and
//     read by all 4 waves — the only operand the waves share;
//   * X fragments (A operand, <= 256 x K bf16, L2-resident) go straight to VGPRs, one block ahead;
//     SWIGLU=true reads the fused gate|up output [M, 2K] and forms silu(g)*u in registers;
//   * split-K over grid.y with the in-launch last-arriver reduction (write-through f32 partials,
//     relaxed ticket, cdna_hip_programming.md Guideline 16 R1) -> one launch, graph-capturable;
//   * epilogue through LDS so Y is written as 16-B row vectors.
// MFMA v_mfma_f32_16x16x32_bf16: A = X rows (row lane&15, k 8(lane>>4)+j), B = W rows (same
// pattern), C row (lane>>4)*4+r, col lane&15.
#include "common.h"

namespace {
constexpr int KB = 64;          // k per pipeline stage
constexpr int LROW = KB + 8;    // LDS row stride in bf16 (144 B: 16-B reads spread over banks)

template <int MT, int NT, bool SWIGLU>
__global__ void __launch_bounds__(256) mm_kernel(const u16* __restrict__ X, long ldx, const u16* __restrict__ W,
                                                 u16* __restrict__ Y, long ldy, int M, int N, int K, int kchunk,
                                                 float* __restrict__ part, int* __restrict__ counters) {
  constexpr int BN = 16 * NT, BM = 64 * MT;
  constexpr int W_BYTES = 2 * BN * LROW * 2, O_BYTES = BM * BN * 2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[W_BYTES > O_BYTES ? W_BYTES : O_BYTES];
  __shared__ int s_last;
  u16(*sW)[BN][LROW] = reinterpret_cast<u16(*)[BN][LROW]>(smem);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rl = lane & 15, kq = 8 * (lane >> 4);
  const int tile = blockIdx.x, split = blockIdx.y, S = gridDim.y;
  const int col0 = tile * BN;
  const int kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
  const int nkb = kend > kbeg ? (kend - kbeg) / KB : 0;

  // W staging: thread t copies row t/4 (of BN <= 64), 16 bf16 at k offset 16 (t%4); NT < 4 uses
  // fewer threads.
  const int wr = threadIdx.x >> 2, wc = (threadIdx.x & 3) * 16;
  const bool w_active = wr < BN;
  const int wn = min(col0 + wr, N - 1);
  const u16* wsrc = W + (long)wn * K + wc;

  // A fragments: MT row groups of this wave
  const u16* arow[MT];
  bool aok[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int r = 16 * MT * wave + 16 * m + rl;
    aok[m] = r < M;
    arow[m] = X + (long)(aok[m] ? r : 0) * ldx + kq;
  }

  f32x4 acc[MT][NT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int AU = SWIGLU ? 2 : 1;
  uint4 wreg[2];
  uint4 a0[2][MT][AU], a1[2][MT][AU];  // ping-pong A stages: [k-step][row group][gate/up]
  auto load_w = [&](int kb) {
    if (w_active) {
      wreg[0] = __builtin_bit_cast(uint4, ldnt_bf16x8(wsrc + kb));
      wreg[1] = __builtin_bit_cast(uint4, ldnt_bf16x8(wsrc + kb + 8));
    }
  };
  auto store_w = [&](int buf) {
    if (w_active) {
      *reinterpret_cast<uint4*>(&sW[buf][wr][wc]) = wreg[0];
      *reinterpret_cast<uint4*>(&sW[buf][wr][wc + 8]) = wreg[1];
    }
  };
  auto load_a = [&](uint4 (&dst)[2][MT][AU], int kb) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        dst[s][m][0] = ld16(arow[m] + kb + 32 * s);
        if constexpr (SWIGLU) dst[s][m][AU - 1] = ld16(arow[m] + K + kb + 32 * s);
      }
  };
  auto compute = [&](const uint4 (&ab)[2][MT][AU], int buf) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[MT], bfr[NT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        uint4 v = ab[s][m][0];
        if constexpr (SWIGLU) {
          float gt[8], up[8];
          unpack8(v, gt);
          unpack8(ab[s][m][AU - 1], up);
#pragma unroll
          for (int j = 0; j < 8; ++j) gt[j] = gt[j] / (1.f + __expf(-gt[j])) * up[j];
          v = pack8(gt);
        }
        if (!aok[m]) v = make_uint4(0, 0, 0, 0);
        af[m] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int n = 0; n < NT; ++n)
        bfr[n] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(&sW[buf][16 * n + rl][32 * s + kq]));
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
    }
  };

  // two k-blocks per trip so both A stages are compile-time arrays (no scratch); the next block's
  // W and A loads are in flight during this block's MFMAs
  if (nkb > 0) {
    load_w(kbeg);
    load_a(a0, kbeg);
    store_w(0);
    __syncthreads();
    for (int i = 0; i < nkb; i += 2) {
      if (i + 1 < nkb) {
        load_w(kbeg + (i + 1) * KB);
        load_a(a1, kbeg + (i + 1) * KB);
      }
      compute(a0, 0);
      if (i + 1 < nkb) store_w(1);
      __syncthreads();
      if (i + 1 < nkb) {
        if (i + 2 < nkb) {
          load_w(kbeg + (i + 2) * KB);
          load_a(a0, kbeg + (i + 2) * KB);
        }
        compute(a1, 1);
        if (i + 2 < nkb) store_w(0);
        __syncthreads();
      }
    }
  }

  // ---- epilogue
  const int rows_here = BM;
  if (S == 1) {
    u16(*sO)[BN] = reinterpret_cast<u16(*)[BN]>(smem);  // W buffers are dead after the last barrier
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          sO[16 * MT * wave + 16 * m + 4 * (lane >> 4) + r][16 * n + rl] = f2bf(acc[m][n][r]);
    __syncthreads();
    constexpr int CPR = BN / 8;  // 16-B chunks per row
    for (int e = threadIdx.x; e < rows_here * CPR; e += 256) {
      const int row = e / CPR, c = (e % CPR) * 8;
      if (row < M && col0 + c < N) st16(Y + (long)row * ldy + col0 + c, *reinterpret_cast<const uint4*>(&sO[row][c]));
    }
    return;
  }
  // split-K partials, column-major per tile: part[split][tile][col][row] (a lane's 4 rows contiguous)
  const long slab = (long)BN * BM;
  const __amdgpu_buffer_rsrc_t pr =
      make_rsrc(part, (unsigned)min((long)gridDim.x * gridDim.y * slab * 4, 0x7fffffffL));
  const long my = ((long)split * gridDim.x + tile) * slab;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int row = 16 * MT * wave + 16 * m + 4 * (lane >> 4), c = 16 * n + rl;
      st_wt16(pr, (unsigned)((my + (long)c * BM + row) * 4),
              make_float4(acc[m][n][0], acc[m][n][1], acc[m][n][2], acc[m][n][3]));
    }
  if (!ticket_last(&counters[tile], S, &s_last)) return;
  u16(*sO)[BN] = reinterpret_cast<u16(*)[BN]>(smem);
  for (int e = threadIdx.x; e < BN * (BM / 4); e += 256) {
    const int c = e / (BM / 4), row = (e % (BM / 4)) * 4;
    float4 v = {0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < S; ++sp) {
      const float4 q = ld_wt16(pr, (unsigned)(((((long)sp * gridDim.x + tile) * slab) + (long)c * BM + row) * 4));
      v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
    }
    sO[row][c] = f2bf(v.x);
    sO[row + 1][c] = f2bf(v.y);
    sO[row + 2][c] = f2bf(v.z);
    sO[row + 3][c] = f2bf(v.w);
  }
  __syncthreads();
  constexpr int CPR = BN / 8;
  for (int e = threadIdx.x; e < rows_here * CPR; e += 256) {
    const int row = e / CPR, c = (e % CPR) * 8;
    if (row < M && col0 + c < N) st16(Y + (long)row * ldy + col0 + c, *reinterpret_cast<const uint4*>(&sO[row][c]));
  }
}

template <int MT, int NT, bool SW>
int launch(const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K, int splits, float* part,
           int* counters, hipStream_t st) {
  const int tiles = (N + 16 * NT - 1) / (16 * NT);
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + KB - 1) / KB * KB;
  const int S = (K + kchunk - 1) / kchunk;
  hipLaunchKernelGGL((mm_kernel<MT, NT, SW>), dim3(tiles, S), dim3(256), 0, st, (const u16*)X, ldx, (const u16*)W,
                     (u16*)Y, ldy, M, N, K, kchunk, part, counters);
  return (int)hipGetLastError();
}

template <int MT, bool SW>
int by_nt(int nt, const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K, int splits,
          float* part, int* counters, hipStream_t st) {
  switch (nt) {
    case 2: return launch<MT, 2, SW>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
    case 4: return launch<MT, 4, SW>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
    default: return -10;
  }
}

template <bool SW>
int by_mt(int M, int nt, const void* X, long ldx, const void* W, void* Y, long ldy, int N, int K, int splits,
          float* part, int* counters, hipStream_t st) {
  if (M <= 64) return by_nt<1, SW>(nt, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  if (M <= 128) return by_nt<2, SW>(nt, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  if (M <= 256) return by_nt<4, SW>(nt, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  return -11;
}
}  // namespace

// part: >= splits * ceil(N / (16 nt)) * 16 nt * BM floats (BM = 64, 128 or 256 by M); counters >= tiles.
extern "C" int dllm_mm_gemm(const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K, int nt,
                            int splits, int swiglu, float* part, int* counters, hipStream_t stream) {
  if (K % KB != 0 || M <= 0 || M > 256 || N % 8 != 0 || splits < 1 || ldy % 8 != 0) return -1;
  if (splits > 1 && (!part || !counters)) return -2;
  return swiglu ? by_mt<true>(M, nt, X, ldx, W, Y, ldy, N, K, splits, part, counters, stream)
                : by_mt<false>(M, nt, X, ldx, W, Y, ldy, N, K, splits, part, counters, stream);
}
