// Small-batch decode GEMV  Y[M, N] = X[M, K] . W[N, K]^T,  M <= 8, optional fused SwiGLU on X.
//
// At M <= 8 a decode projection is a pure weight stream (2-8 FMAs per weight element, VALU rate
// is ~30x above what HBM can feed), so this kernel is shaped for bytes in flight, not for MFMA:
//   * each wave owns R output columns (= R rows of W) and streams them along K with fully
//     contiguous 1 KB wave-instructions (lane l reads W[n][k + 8l .. k + 8l + 7]; the MFMA
//     fragment layout of the skinny kernel splits a row into 64-B pieces instead);
//   * a wave issues UNR x R such loads before its first FMA (16-64 KB in flight per CU at
//     8 waves/CU), the 'GEMV / M <= 16' row of the staging table: W goes straight to VGPRs;
//   * batch 1 (XG): X is loaded with every W trip (16 B per lane beside each 1 KB W piece, L1 / L2
//     hits) - no LDS stage, no barrier before the first FMA (measured 0.2-1 us faster per GEMV);
//   * batch 2-8: X is staged once per workgroup into LDS (M x K bf16 <= 64 KB) while the first W trip is in
//     flight, then read with conflict-free ds_read_b128 (per-iteration L2 reads of X measured
//     slow: a dependent L2 round trip per k-step); with SWIGLU, X is the fused gate|up output
//     [M, 2K] and silu(gate) * up is formed in the staging pass (the down projection absorbs the
//     activation kernel);
//   * the next W trip is issued before the current one is consumed (register double buffer);
//   * NORM: the pre-projection RMSNorm (+ residual add) runs in the staging pass, so a decode
//     layer at batch <= 8 drops both norm launches (norm.hip) from its chain;
//   * f32 FMA, one 64-lane butterfly reduction per (row, column) at the end; no split-K, no
//     workspace, no inter-workgroup traffic: one launch per projection, graph-capturable.
//   * EPI (fused decoder-layer epilogues, the GEMV twin of tgemm.hip's): at batch <= 8 a
//     standalone epilogue kernel (qkv_post / res_add_ssq / swiglu_post) costs as much as the GEMV
//     itself (one ~4 us launch each, profiles/r2_decode_replay_b1.md), so the GEMV applies them:
//       EPI_RESADD : r[m, n] = bf16(bf16(acc) + r[m, n]) in place, and the workgroup's partial
//                    row sums of r^2 into ssq_out[blockIdx.x][m] (one slot per workgroup);
//       EPI_QKV    : row scale rinv[m] from the producer's partial sums (folded RMSNorm), RoPE on
//                    the (c, c + 16) pairs of the permuted q/k rows, q out, K and V^T written
//                    straight into the paged caches;
//       EPI_SWIGLU : act = silu(g * rinv) * (u * rinv) for the interleaved 16-gate/16-up rows.
//     QKV / SWIGLU need both members of a (c, c + 16) pair in one workgroup, so those modes map
//     columns "paired": waves 0-1 take first-half columns of a 32-column group, waves 2-3 the
//     matching second-half ones; the accumulators meet in LDS for the epilogue.  rinv is summed
//     from the partials while the first W trip is in flight (no extra latency on the chain).
// Chosen per (M, N, K) by the host autotuner (ops.gemm) only where it beats the other plans.
#include "common.h"

#include <algorithm>

namespace {

enum { GV_PLAIN = 0, GV_RESADD = 1, GV_QKV = 2, GV_SWIGLU = 3 };

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// acc + x.lo * w.lo + x.hi * w.hi for two packed bf16 pairs (v_dot2c_f32_bf16)
__device__ __forceinline__ float dot2bf(uint32_t x, uint32_t w, float acc) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, x), __builtin_bit_cast(bf16x2, w), acc, false);
}

struct EpiArgs {                 // fused output epilogues (EPI != GV_PLAIN)
  u16* res;                      // RESADD: residual stream [M, ldr], updated in place
  long ldr;
  float* ssq_out;                // RESADD: partial row sums of r^2, [gridDim.x][ssq_out_ld]
  long ssq_out_ld;
  const float* ssq_in;           // QKV / SWIGLU: producer partial sums [ssq_n][ssq_in_ld]
  int ssq_n;
  long ssq_in_ld;
  float scale, eps;              // rinv = rsqrt(sum * scale + eps)
  const int* pos;                // QKV: positions, cos|sin table [*, d], cache slots (-1: no write)
  const float* cos_sin;
  const int* slots;
  u16* q_out;                    // QKV: q [M, nq, d]; kc [blocks, nkv, 16, d]; vc [blocks, nkv, d, 16]
  u16* kc;
  u16* vc;
  int nq, nkv, d;
};

struct NormArgs {         // NORM: X is the sub-layer output h; the kernel forms r = h + res_in (bf16),
  const u16* res_in;     // workgroup 0 stores r to res_out (a different buffer: every workgroup
  u16* res_out;          // reads res_in), and the GEMV input is rmsnorm(r) * w  (norm.hip numerics)
  const u16* w;
  float eps;
};

__host__ __device__ constexpr unsigned gemv_blocks_rt(int N, int R) { return (unsigned)((N + 4 * R - 1) / (4 * R)); }

template <int M, int R, int UNR, bool SWIGLU, bool NORM, int EPI, bool XG = false>
__global__ void __launch_bounds__(256) gemv_kernel(const u16* __restrict__ X, long ldx, const u16* __restrict__ W,
                                                   u16* __restrict__ Y, long ldy, int N, int K, NormArgs na,
                                                   EpiArgs ea) {
  extern __shared__ uint4 xs_raw[];  // X (SwiGLU applied) staged once per workgroup: [M][K] bf16
  u16* xs = reinterpret_cast<u16*>(xs_raw);
  // epilogue scratch after X (and NORM's reduction slots): rinv [M], accumulators [4][R][M],
  // per-wave row sums [4][M]
  float* s_ri = reinterpret_cast<float*>(xs + (XG ? 0L : (long)M * K)) + (NORM ? 4 * M : 0);
  float* s_ep = s_ri + M;
  float* s_red = s_ep + 4 * R * M;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr bool PAIRED = EPI == GV_QKV || EPI == GV_SWIGLU;
  // Virtual blocks: the launch may cap the grid below the column blocks (gemv_grid), and then a
  // workgroup walks blocks vb, vb + gridDim.x, ... with X staged ONCE: at batch 2-8 a per-block
  // X stage moved as many bytes from L2 as the weights themselves (M x K per 4R columns)
  const int nvb = (int)gemv_blocks_rt(N, R);
  auto col0 = [&](int vb) {
    if constexpr (PAIRED) {
      // 8/R blocks per 32-column group; each takes 2R first-half columns (waves 0, 1) and the
      // 2R second-half columns 16 further on (waves 2, 3)
      constexpr int PER = 8 / R;
      const int g = vb / PER, j0 = (vb % PER) * 2 * R;
      return g * 32 + (wave >> 1) * 16 + j0 + (wave & 1) * R;
    } else {
      return (vb * 4 + wave) * R;
    }
  };
  int vb = blockIdx.x;
  int n0 = col0(vb);
  bool active = n0 < N;  // inactive waves still stage X and pass the barriers
  const u16* wr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) wr[r] = W + (long)min(n0 + r, N - 1) * K;

  constexpr int STEP = 512;  // K elements per wave-instruction
  constexpr int TRIP = STEP * UNR;
  uint4 w[UNR][R], wn[UNR][R];
  // XG (batch 1, plain X): X travels with W in every trip (L1/L2 hits, no LDS stage, no barrier)
  uint4 xg[XG ? UNR : 1][XG ? M : 1], xgn[XG ? UNR : 1][XG ? M : 1];
#define DLLM_GEMV_LOAD(DST, XDST, KB, ROWS, ACT)                                                     \
  _Pragma("unroll") for (int u = 0; u < UNR; ++u) {                                                 \
    const int k_ = (KB) + u * STEP + 8 * lane;                                                      \
    _Pragma("unroll") for (int r = 0; r < R; ++r) DST[u][r] =                                       \
        ((ACT) && k_ < K) ? __builtin_bit_cast(uint4, ldnt_bf16x8(ROWS[r] + k_)) : make_uint4(0, 0, 0, 0); \
    if constexpr (XG) {                                                                             \
      _Pragma("unroll") for (int m = 0; m < M; ++m) XDST[u][m] =                                    \
          ((ACT) && k_ < K) ? ld16(X + (long)m * ldx + k_) : make_uint4(0, 0, 0, 0);                \
    }                                                                                               \
  }
  DLLM_GEMV_LOAD(w, xg, 0, wr, active)  // the first trip of W is in flight while X is staged
  if constexpr (PAIRED) {
    // folded RMSNorm row scale: lane-parallel sum of the producer's partial sums, wave w -> rows w, w + 4
    // (a GEMV producer leaves one slot per workgroup, e.g. 512 at N = 2048: 8 independent loads
    // per lane are issued before the first add, so the sum costs one L2 round trip, not eight;
    // requesting them ahead of the weight stream instead measured no different, round 4)
    for (int m = wave; m < M; m += 4) {
      float sacc = 0.f;
      for (int i0 = 0; i0 < ea.ssq_n; i0 += 512) {
        float part[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = i0 + u * 64 + lane;
          part[u] = i < ea.ssq_n ? ea.ssq_in[(long)i * ea.ssq_in_ld + m] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) sacc += part[u];
      }
      sacc = wave_sum(sacc);
      if (lane == 0) s_ri[m] = rsqrtf(sacc * ea.scale + ea.eps);
    }
  }
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
  } else if constexpr (!XG) {
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
  if constexpr (!XG) __syncthreads();

  float v2sum = 0.f;  // RESADD: this lane's row sums of r^2 over the workgroup's blocks
  for (;;) {
  const int vn = vb + (int)gridDim.x;  // the workgroup's next block (its first W trip overlaps this one)
  const int n0n = vn < nvb ? col0(vn) : N;
  const bool activen = n0n < N;
  const u16* wrn[R];
#pragma unroll
  for (int r = 0; r < R; ++r) wrn[r] = W + (long)min(n0n + r, N - 1) * K;
  float acc[M][R];
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[m][r] = 0.f;
  for (int kb = 0; kb < K; kb += TRIP) {
    // next trip in flight during this one: this block's, else the next block's first
    if (kb + TRIP < K) {
      DLLM_GEMV_LOAD(wn, xgn, kb + TRIP, wr, active)
    } else if (vn < nvb) {
      DLLM_GEMV_LOAD(wn, xgn, 0, wrn, activen)
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int k = kb + u * STEP + 8 * lane;
      if (k < K) {
        // packed bf16 dot products (v_dot2c_f32_bf16: two exact bf16 products added into the f32
        // accumulator, no unpacking): 4 VALU ops per (row, column, 16-B piece) instead of 8 FMAs plus
        // 16 conversions - at 8 rows the unpacked form was VALU-bound (8.5 ops per weight byte)
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const uint4 xv = XG ? xg[u][m] : ld16(xs + (long)m * K + k);
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const uint4 wv = w[u][r];
            float a = acc[m][r];
            a = dot2bf(xv.x, wv.x, a);
            a = dot2bf(xv.y, wv.y, a);
            a = dot2bf(xv.z, wv.z, a);
            a = dot2bf(xv.w, wv.w, a);
            acc[m][r] = a;
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
#pragma unroll
      for (int r = 0; r < R; ++r) w[u][r] = wn[u][r];
      if constexpr (XG) {
#pragma unroll
        for (int m = 0; m < M; ++m) xg[u][m] = xgn[u][m];
      }
    }
  }
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float v = acc[m][r];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      acc[m][r] = v;
    }
  if constexpr (EPI == GV_PLAIN) {
    if (active && lane == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (n0 + r >= N) break;
#pragma unroll
        for (int m = 0; m < M; ++m) Y[(long)m * ldy + n0 + r] = f2bf(acc[m][r]);
      }
    }
  } else if constexpr (EPI == GV_RESADD) {
    // r = bf16(bf16(acc) + r) (res_add_ssq numerics), summed into this lane's r^2.  Lane (m, r) =
    // (lane / R, lane % R) owns one output, so a wave's residual read-modify-writes go out together
    // (one round trip, not M x R dependent ones from lane 0); after the butterfly every lane holds
    // every acc[m][r].
    if (active && lane < M * R) {
      const int lm = lane / R, lr = lane % R;
      float a = 0.f;
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (m == lm && r == lr) a = acc[m][r];
      if (n0 + lr < N) {
        u16* p = ea.res + (long)lm * ea.ldr + n0 + lr;
        const float v = bf2f(f2bf(bf2f(f2bf(a)) + bf2f(*p)));
        *p = f2bf(v);
        v2sum += v * v;
      }
    }
  } else {
    // paired modes: accumulators meet in LDS, thread (p, m) owns pair p of row m
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int m = 0; m < M; ++m) s_ep[(wave * R + r) * M + m] = acc[m][r];
    }
    __syncthreads();
    if (threadIdx.x < 2 * R * M) {
      constexpr int PER = 8 / R;
      const int m = threadIdx.x % M, p = threadIdx.x / M;
      const int g = vb / PER, j = (vb % PER) * 2 * R + p;  // column offset in the group
      const float x1 = s_ep[p * M + m], x2 = s_ep[(2 * R + p) * M + m];      // columns 32g + j, + 16
      const float ri = s_ri[m];
      if constexpr (EPI == GV_SWIGLU) {
        const float gv = bf2f(f2bf(x1 * ri)), uv = bf2f(f2bf(x2 * ri));
        Y[(long)m * ldy + 16 * g + j] = f2bf(gv / (1.f + __expf(-gv)) * uv);
      } else {
        const int d = ea.d, hd = d / 2, qcols = ea.nq * d, kcols = ea.nkv * d;
        const int c = 32 * g + j, slot = ea.slots[m];
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
    if (vn < nvb) __syncthreads();  // s_ep is rewritten by the next block (uniform condition)
  }
  if (vn >= nvb) break;
  vb = vn;
  n0 = n0n;
  active = activen;
#pragma unroll
  for (int r = 0; r < R; ++r) wr[r] = wrn[r];
  }
#undef DLLM_GEMV_LOAD
  if constexpr (EPI == GV_RESADD) {
    // this workgroup's partial row sums of r^2 over all its blocks: one slot per workgroup
#pragma unroll
    for (int o = 1; o < R; o <<= 1) v2sum += __shfl_xor(v2sum, o, 64);  // the R lanes of a row (aligned groups)
    if (lane < M * R && lane % R == 0) s_red[wave * M + lane / R] = v2sum;  // inactive waves store zeros
    __syncthreads();
    if (threadIdx.x < M) {
      const int m = threadIdx.x;
      ea.ssq_out[(long)blockIdx.x * ea.ssq_out_ld + m] = s_red[m] + s_red[M + m] + s_red[2 * M + m] + s_red[3 * M + m];
    }
  }
}

template <int R>
constexpr unsigned gemv_blocks(int N) { return gemv_blocks_rt(N, R); }

// Grid of a batch 2-8 launch with N >= g_grid_nmin: at most max(g_grid_min, N / (g_grid_xdiv M))
// workgroups, so the X bytes every workgroup stages (M x K) stay <= 1 / g_grid_xdiv of the weight
// bytes.  Batch 1 (X rides with W, no stage), narrower N and g_grid_xdiv = 0 keep one workgroup per
// column block.  Measured (profiles/r6_small_batch.md, scripts/exp/gemv_probe.py): the cap takes
// 7-27 % off the wide gate|up projections at batch 2-8 and costs 5-35 % on the narrow ones
// (QKV / Wo / down), whose grids it would shrink below the CU count's worth of bytes in flight.
int g_grid_min = 512, g_grid_xdiv = 4, g_grid_nmin = 8192;
unsigned gemv_grid(int M, int N, int R) {
  const unsigned nvb = gemv_blocks_rt(N, R);
  if (M == 1 || g_grid_xdiv <= 0 || N < g_grid_nmin) return nvb;
  const unsigned want = (unsigned)std::max(g_grid_min, (N + g_grid_xdiv * M - 1) / (g_grid_xdiv * M));
  return std::min(nvb, want);
}

template <int M, int R, bool SW, bool NORM, int EPI>
void launch_gemv(const void* x, long ldx, const void* w, void* y, long ldy, int N, int K, const NormArgs& na,
                 const EpiArgs& ea, hipStream_t stream) {
  // XG (batch 1, plain X): X rides along in every W trip (L1 / L2 hits) instead of an LDS stage
  // and barrier.  Measured at batch 1 (scripts/exp/gemv_probe.py, profiles/r4_single_stream.md):
  // 0.2-0.6 us off TinyLlama's fused QKV / Wo / gate|up / down GEMVs and up to 1 us off
  // Llama-3-8B's, never slower; at batch 2 it is slower on the large shapes, so batch 1 only.
  if constexpr (M == 1 && !SW && !NORM) {
    const size_t lds_xg = EPI != GV_PLAIN ? (size_t)(M + 4 * R * M + 4 * M) * sizeof(float) : 0;
    hipLaunchKernelGGL((gemv_kernel<M, R, 4, SW, NORM, EPI, true>), dim3(gemv_blocks<R>(N)), dim3(256), lds_xg,
                       stream, (const u16*)x, ldx, (const u16*)w, (u16*)y, ldy, N, K, na, ea);
    return;
  }
  const size_t lds = (size_t)M * K * 2 + (NORM ? 4 * M * sizeof(float) : 0) +
                     (EPI != GV_PLAIN ? (size_t)(M + 4 * R * M + 4 * M) * sizeof(float) : 0);
  // Long rows on a small grid at batch 1-2 (TinyLlama's down projection: K = 5632 is 11
  // wave-loads per row, N = 2048 is 512 workgroups, 2 per CU): with 4 loads per trip a wave waits
  // out three dependent HBM latencies; 8 / 12 per trip put a whole row of up to 4096 / 6144
  // elements in flight at once (64 / 96 VGPRs of W buffers).  Measured (1x MI355X, B = 1 decode
  // step): TinyLlama 0.890 -> 0.872-0.883 ms; on larger grids (Llama-3-8B, >= 1024 workgroups) the
  // lower occupancy cost ~1 %, so they keep 4-load trips.
  if constexpr (M <= 2 && R == 1) {
    if (K > 2048 && K <= 6144 && gemv_blocks<R>(N) <= 512) {
      if (K <= 4096)
        hipLaunchKernelGGL((gemv_kernel<M, R, 8, SW, NORM, EPI>), dim3(gemv_grid(M, N, R)), dim3(256), lds, stream,
                           (const u16*)x, ldx, (const u16*)w, (u16*)y, ldy, N, K, na, ea);
      else
        hipLaunchKernelGGL((gemv_kernel<M, R, 12, SW, NORM, EPI>), dim3(gemv_grid(M, N, R)), dim3(256), lds, stream,
                           (const u16*)x, ldx, (const u16*)w, (u16*)y, ldy, N, K, na, ea);
      return;
    }
  }
  constexpr int UNR = M <= 4 ? 4 : 2;
  hipLaunchKernelGGL((gemv_kernel<M, R, UNR, SW, NORM, EPI>), dim3(gemv_grid(M, N, R)), dim3(256), lds, stream,
                     (const u16*)x, ldx, (const u16*)w, (u16*)y, ldy, N, K, na, ea);
}

template <int M, bool SW, bool NORM, int EPI>
int dispatch_r(int R, const void* x, long ldx, const void* w, void* y, long ldy, int N, int K, const NormArgs& na,
               const EpiArgs& ea, hipStream_t s) {
  switch (R) {
    case 1: launch_gemv<M, 1, SW, NORM, EPI>(x, ldx, w, y, ldy, N, K, na, ea, s); break;
    case 2: launch_gemv<M, 2, SW, NORM, EPI>(x, ldx, w, y, ldy, N, K, na, ea, s); break;
    case 4: launch_gemv<M, 4, SW, NORM, EPI>(x, ldx, w, y, ldy, N, K, na, ea, s); break;
    default: return -2;
  }
  return 0;
}

template <bool SW, bool NORM, int EPI>
int dispatch_m(int Mp, int R, const void* x, long ldx, const void* w, void* y, long ldy, int N, int K,
               const NormArgs& na, const EpiArgs& ea, hipStream_t s) {
  switch (Mp) {
    case 1: return dispatch_r<1, SW, NORM, EPI>(R, x, ldx, w, y, ldy, N, K, na, ea, s);
    case 2: return dispatch_r<2, SW, NORM, EPI>(R, x, ldx, w, y, ldy, N, K, na, ea, s);
    case 4: return dispatch_r<4, SW, NORM, EPI>(R, x, ldx, w, y, ldy, N, K, na, ea, s);
    case 8: return dispatch_r<8, SW, NORM, EPI>(R, x, ldx, w, y, ldy, N, K, na, ea, s);
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
  const EpiArgs ea{};
  int rc;
  if (norm)
    rc = dispatch_m<false, true, GV_PLAIN>(M, R, x, ldx, w, y, ldy, N, K, na, ea, stream);
  else if (swiglu)
    rc = dispatch_m<true, false, GV_PLAIN>(M, R, x, ldx, w, y, ldy, N, K, na, ea, stream);
  else
    rc = dispatch_m<false, false, GV_PLAIN>(M, R, x, ldx, w, y, ldy, N, K, na, ea, stream);
  if (rc) return rc;
  return (int)hipGetLastError();
}

// Number of partial row-sum slots a GV_RESADD launch of M x N writes (one per workgroup).
extern "C" int dllm_gemv_slots(int M, int N, int R) {
  return (R == 1 || R == 2 || R == 4) ? (int)gemv_grid(M, N, R) : -1;
}

// Grid policy of the batch 2-8 launches (gemv_grid); xdiv 0 = one workgroup per column block.
// Set before any graph capture: a captured launch keeps the grid it was captured with.
extern "C" void dllm_gemv_set_grid(int min_blocks, int xdiv, int n_min) {
  g_grid_min = min_blocks > 0 ? min_blocks : 1;
  g_grid_xdiv = xdiv;
  g_grid_nmin = n_min;
}

// GEMV with a fused decoder epilogue (epi: 1 RESADD, 2 QKV, 3 SWIGLU; see the header).
//   RESADD: res[M, N] += x . w^T (y unused), partial row sums of res^2 -> ssq_out[slot][m]
//   QKV   : w = the permuted/folded QKV weight, N = (nq + 2 nkv) d; q_out / kc / vc as qkv_post
//   SWIGLU: w = interleaved gate|up rows (N = 2I), y = act [M, I]
// Host contract (csrc/bindings.cpp checks it): M in {1, 2, 4, 8}, R in {1, 2, 4}, K % 8 == 0,
// M x K x 2 B <= 64 KB, N % 32 == 0 for QKV / SWIGLU (and d % 32 == 0 for QKV), ssq_out rows >=
// dllm_gemv_slots(M, N, R) for RESADD.
extern "C" int dllm_gemv_epi(const void* x, long ldx, const void* w, void* y, long ldy, int M, int N, int K, int R,
                             int epi, void* res, long ldr, float* ssq_out, long ssq_out_ld, const float* ssq_in,
                             int ssq_n, long ssq_in_ld, float scale, float eps, const int* pos, const float* cos_sin,
                             const int* slots, void* q_out, void* kc, void* vc, int nq, int nkv, int d,
                             hipStream_t stream) {
  if (K % 8 != 0 || N <= 0 || (long)M * K * 2 > GEMV_MAX_LDS) return -3;
  if ((epi == GV_QKV || epi == GV_SWIGLU) && (N % 32 || !ssq_in || ssq_n < 1)) return -4;
  if (epi == GV_QKV && (d % 32 || N != (nq + 2 * nkv) * d || !q_out || !kc || !vc || !pos || !cos_sin || !slots))
    return -5;
  if (epi == GV_RESADD && (!res || !ssq_out || ldr % 8)) return -6;
  const NormArgs na{};
  const EpiArgs ea{(u16*)res, ldr, ssq_out, ssq_out_ld, ssq_in, ssq_n, ssq_in_ld, scale, eps, pos, cos_sin, slots,
                   (u16*)q_out, (u16*)kc, (u16*)vc, nq, nkv, d};
  int rc;
  switch (epi) {
    case GV_RESADD: rc = dispatch_m<false, false, GV_RESADD>(M, R, x, ldx, w, y, ldy, N, K, na, ea, stream); break;
    case GV_QKV: rc = dispatch_m<false, false, GV_QKV>(M, R, x, ldx, w, y, ldy, N, K, na, ea, stream); break;
    case GV_SWIGLU: rc = dispatch_m<false, false, GV_SWIGLU>(M, R, x, ldx, w, y, ldy, N, K, na, ea, stream); break;
    default: return -7;
  }
  if (rc) return rc;
  return (int)hipGetLastError();
}
