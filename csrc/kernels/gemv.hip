// Small-batch decode GEMV  Y[M, N] = X[M, K] . W[N, K]^T,  M <= 8, optional fused SwiGLU on X.
//
// At M <= 8 a decode projection is a pure weight stream (2-8 FMAs per weight element, VALU rate
// is ~30x above what HBM can feed), so this kernel is shaped for bytes in flight, not for MFMA:
//   * each wave owns R output columns (= R rows of W) and streams them along K with fully
//     contiguous 1 KB wave-instructions (lane l reads W[n][k + 8l .. k + 8l + 7]; the MFMA
//     fragment layout of the skinny kernel splits a row into 64-B pieces instead);
//   * a wave issues UNR x R such loads before its first FMA (16-64 KB in flight per CU at
//     8 waves/CU), the 'GEMV / M <= 16' row of the staging table: W goes straight to VGPRs;
//   * X is staged once per workgroup into LDS (M x K bf16 <= 64 KB) while the first W trip is in
//     flight, then read with conflict-free ds_read_b128 (per-iteration L2 reads of X measured
//     slow: a dependent L2 round trip per k-step); with SWIGLU, X is the fused gate|up output
//     [M, 2K] and silu(gate) * up is formed in the staging pass (the down projection absorbs the
//     activation kernel);
//   * the next W trip is issued before the current one is consumed (register double buffer);
//   * NORM: the pre-projection RMSNorm (+ residual add) runs in the staging pass, so a decode
//     layer at batch <= 8 drops both norm launches (norm.hip) from its chain;
//   * f32 FMA, one 64-lane butterfly reduction per (row, column) at the end; no split-K, no
//     workspace, no inter-workgroup traffic: one launch per projection, graph-capturable.
// Chosen per (M, N, K) by the host autotuner (ops.gemm) only where it beats the other plans.
#include "common.h"

namespace {

struct NormArgs {         // NORM: X is the sub-layer output h; the kernel forms r = h + res_in (bf16),
  const u16* res_in;     // workgroup 0 stores r to res_out (a different buffer: every workgroup
  u16* res_out;          // reads res_in), and the GEMV input is rmsnorm(r) * w  (norm.hip numerics)
  const u16* w;
  float eps;
};

template <int M, int R, int UNR, bool SWIGLU, bool NORM>
__global__ void __launch_bounds__(256) gemv_kernel(const u16* __restrict__ X, long ldx, const u16* __restrict__ W,
                                                   u16* __restrict__ Y, long ldy, int N, int K, NormArgs na) {
  extern __shared__ uint4 xs_raw[];  // X (SwiGLU applied) staged once per workgroup: [M][K] bf16
  u16* xs = reinterpret_cast<u16*>(xs_raw);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * 4 + wave) * R;
  const bool active = n0 < N;  // inactive waves still stage X and pass the barrier
  const u16* wr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) wr[r] = W + (long)min(n0 + r, N - 1) * K;

  constexpr int STEP = 512;  // K elements per wave-instruction
  constexpr int TRIP = STEP * UNR;
  uint4 w[UNR][R], wn[UNR][R];
#define DLLM_GEMV_LOAD(DST, KB)                                                                      \
  _Pragma("unroll") for (int u = 0; u < UNR; ++u) {                                                 \
    const int k_ = (KB) + u * STEP + 8 * lane;                                                      \
    _Pragma("unroll") for (int r = 0; r < R; ++r) DST[u][r] =                                       \
        (active && k_ < K) ? __builtin_bit_cast(uint4, ldnt_bf16x8(wr[r] + k_)) : make_uint4(0, 0, 0, 0); \
  }
  DLLM_GEMV_LOAD(w, 0)  // the first trip of W is in flight while X is staged
  if constexpr (NORM) {
    float* red = reinterpret_cast<float*>(xs + (long)M * K);  // [4 waves][M]
    float ss[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      ss[m] = 0.f;
      for (int c8 = threadIdx.x; c8 < (K >> 3); c8 += 256) {
        const int c = c8 << 3;
        float a[8], b[8];
        unpack8(ld16(X + (long)m * ldx + c), a);
        unpack8(ld16(na.res_in + (long)m * K + c), b);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] += b[j];
        const uint4 pk = pack8(a);  // the residual stream stays bf16
        if (blockIdx.x == 0) st16(na.res_out + (long)m * K + c, pk);
        st16(xs + (long)m * K + c, pk);
        unpack8(pk, a);
#pragma unroll
        for (int j = 0; j < 8; ++j) ss[m] += a[j] * a[j];
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) ss[m] += __shfl_xor(ss[m], o, 64);
      if (lane == 0) red[wave * M + m] = ss[m];
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float rstd = rsqrtf((red[m] + red[M + m] + red[2 * M + m] + red[3 * M + m]) / K + na.eps);
      for (int c8 = threadIdx.x; c8 < (K >> 3); c8 += 256) {
        const int c = c8 << 3;
        float a[8], g[8];
        unpack8(ld16(xs + (long)m * K + c), a);
        unpack8(ld16(na.w + c), g);
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = a[j] * rstd * g[j];
        st16(xs + (long)m * K + c, pack8(a));  // each thread rewrites only the vectors it wrote
      }
    }
  } else {
  for (int v = threadIdx.x; v < M * (K >> 3); v += 256) {
    const int m = v / (K >> 3), c = (v - m * (K >> 3)) << 3;
    uint4 xv = ld16(X + (long)m * ldx + c);
    if constexpr (SWIGLU) {
      float g[8], up[8];
      unpack8(xv, g);
      unpack8(ld16(X + (long)m * ldx + K + c), up);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = g[j] / (1.f + __expf(-g[j])) * up[j];
      xv = pack8(g);  // bf16, as the unfused silu_mul output the GEMM would read
    }
    st16(xs + (long)m * K + c, xv);
  }
  }
  __syncthreads();

  float acc[M][R];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[m][r] = 0.f;
  for (int kb = 0; kb < K; kb += TRIP) {
    if (kb + TRIP < K) { DLLM_GEMV_LOAD(wn, kb + TRIP) }  // next trip in flight during this one
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int k = kb + u * STEP + 8 * lane;
      if (k < K) {
        float wf[R][8];
#pragma unroll
        for (int r = 0; r < R; ++r) unpack8(w[u][r], wf[r]);
#pragma unroll
        for (int m = 0; m < M; ++m) {
          float xf[8];
          unpack8(ld16(xs + (long)m * K + k), xf);
#pragma unroll
          for (int r = 0; r < R; ++r)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[m][r] = fmaf(xf[j], wf[r][j], acc[m][r]);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
#pragma unroll
      for (int r = 0; r < R; ++r) w[u][r] = wn[u][r];
  }
#undef DLLM_GEMV_LOAD
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float v = acc[m][r];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      acc[m][r] = v;
    }
  if (active && lane == 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (n0 + r >= N) break;
#pragma unroll
      for (int m = 0; m < M; ++m) Y[(long)m * ldy + n0 + r] = f2bf(acc[m][r]);
    }
  }
}

template <int M, int R, bool SW, bool NORM>
void launch_gemv(const void* x, long ldx, const void* w, void* y, long ldy, int N, int K, const NormArgs& na,
                 hipStream_t stream) {
  constexpr int UNR = M <= 2 ? 4 : 2;
  const unsigned blocks = (unsigned)((N + 4 * R - 1) / (4 * R));
  const size_t lds = (size_t)M * K * 2 + (NORM ? 4 * M * sizeof(float) : 0);
  hipLaunchKernelGGL((gemv_kernel<M, R, UNR, SW, NORM>), dim3(blocks), dim3(256), lds, stream, (const u16*)x, ldx,
                     (const u16*)w, (u16*)y, ldy, N, K, na);
}

template <int M, bool SW, bool NORM>
int dispatch_r(int R, const void* x, long ldx, const void* w, void* y, long ldy, int N, int K, const NormArgs& na,
               hipStream_t s) {
  switch (R) {
    case 1: launch_gemv<M, 1, SW, NORM>(x, ldx, w, y, ldy, N, K, na, s); break;
    case 2: launch_gemv<M, 2, SW, NORM>(x, ldx, w, y, ldy, N, K, na, s); break;
    case 4: launch_gemv<M, 4, SW, NORM>(x, ldx, w, y, ldy, N, K, na, s); break;
    default: return -2;
  }
  return 0;
}

template <bool SW, bool NORM>
int dispatch_m(int Mp, int R, const void* x, long ldx, const void* w, void* y, long ldy, int N, int K,
               const NormArgs& na, hipStream_t s) {
  switch (Mp) {
    case 1: return dispatch_r<1, SW, NORM>(R, x, ldx, w, y, ldy, N, K, na, s);
    case 2: return dispatch_r<2, SW, NORM>(R, x, ldx, w, y, ldy, N, K, na, s);
    case 4: return dispatch_r<4, SW, NORM>(R, x, ldx, w, y, ldy, N, K, na, s);
    case 8: return dispatch_r<8, SW, NORM>(R, x, ldx, w, y, ldy, N, K, na, s);
    default: return -1;
  }
}
}  // namespace

constexpr long GEMV_MAX_LDS = 64 * 1024;  // staged X bytes per workgroup (M x K bf16)

// M must be 1, 2, 4 or 8 (the decode buckets below 16; the autotuner offers this kernel only
// for them); K % 8 == 0; M x K x 2 B <= 64 KB; rows of X, W and Y 16-B aligned.
extern "C" int dllm_gemv(const void* x, long ldx, const void* w, void* y, long ldy, int M, int N, int K, int R,
                         int swiglu, const void* res_in, void* res_out, const void* norm_w, float eps,
                         hipStream_t stream) {
  if (K % 8 != 0 || N <= 0 || (long)M * K * 2 > GEMV_MAX_LDS) return -3;
  const bool norm = norm_w != nullptr;
  if (norm && (swiglu || !res_in || !res_out || res_in == res_out || ldx % 8)) return -4;
  const NormArgs na{(const u16*)res_in, (u16*)res_out, (const u16*)norm_w, eps};
  int rc;
  if (norm)
    rc = dispatch_m<false, true>(M, R, x, ldx, w, y, ldy, N, K, na, stream);
  else if (swiglu)
    rc = dispatch_m<true, false>(M, R, x, ldx, w, y, ldy, N, K, na, stream);
  else
    rc = dispatch_m<false, false>(M, R, x, ldx, w, y, ldy, N, K, na, stream);
  if (rc) return rc;
  return (int)hipGetLastError();
}
