// Decode GEMM, variant B:  Y[M, N] = X[M, K] . W[N, K]^T  for 16 < M <= 128 (+ fused SwiGLU).
//
// Variant A (skinny_gemm.hip) gives every wave its own K range, so every wave re-reads X from
// L2: X traffic / W traffic = M / (16 NTW) — at M = 64 the activations cost more than the weights.
// Here the 4 waves of a workgroup own DIFFERENT columns over the SAME K range, and X is staged
// once per workgroup into LDS in 256-wide K chunks (double-buffered, SwiGLU applied while
// staging), so X costs 1/NTW of W from L2 and the weight stream — the actual HBM traffic —
// runs with a register prefetch of the next chunk's 8 k-steps (two register stages).
//   workgroup tile: 64*NTW columns x [kbeg, kbeg + kchunk) ; grid.y = split-K, reduced in the
//   kernel by the last-arriving workgroup (same ticket protocol as variant A).
// LDS image: [2][Mp][KC + 8] bf16 (KC = 256, or 128 for Mp >= 64) (16-B row pad: A-fragment ds_read_b128 of 16 rows at one
// k offset spread over all 64 banks).
#include "common.h"

namespace {
constexpr int PAD = 8;

template <int MT, int NTW, bool SWIGLU>
__global__ void __launch_bounds__(256) skinny_lds_kernel(const u16* __restrict__ X, long ldx,
                                                         const u16* __restrict__ W, u16* __restrict__ Y, long ldy,
                                                         int M, int N, int K, int kchunk, float* __restrict__ part,
                                                         int* __restrict__ counters) {
  constexpr int MP = MT * 16;
  constexpr int NC = 64 * NTW;
  constexpr int KC = MT >= 4 ? 128 : 256;  // K chunk staged in LDS (<= 34 KB per buffer pair at MT 4)
  constexpr int KSTEPS = KC / 32;
  __shared__ __attribute__((aligned(16))) u16 xs[2][MP][KC + PAD];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int tile = blockIdx.x, split = blockIdx.y, S = gridDim.y;
  const int col0 = tile * NC + wave * 16 * NTW;
  const int kbeg = split * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const int nch = (kend - kbeg + KC - 1) / KC;

  const u16* wrow[NTW];
#pragma unroll
  for (int n = 0; n < NTW; ++n) {
    int c = col0 + 16 * n + r16;
    c = c < N ? c : N - 1;
    wrow[n] = W + (long)c * K + 8 * g;
  }

  // X chunk -> LDS (16 B per thread per pass), SwiGLU applied on the way
  auto stage = [&](int buf, int k0) {
    const int klen = min(KC, kend - k0);
    for (int e = tid; e < MP * (KC / 8); e += 256) {
      const int row = e / (KC / 8), c8 = (e % (KC / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (row < M && c8 < klen) {
        const u16* src = X + (long)row * ldx + k0 + c8;
        if constexpr (SWIGLU) {
          float gt[8], up[8];
          unpack8(ld16(src), gt);
          unpack8(ld16(src + K), up);
#pragma unroll
          for (int j = 0; j < 8; ++j) gt[j] = gt[j] / (1.f + __expf(-gt[j])) * up[j];
          v = pack8(gt);
        } else {
          v = ld16(src);
        }
      }
      *reinterpret_cast<uint4*>(&xs[buf][row][c8]) = v;
    }
  };
  auto loadw = [&](bf16x8 (&wf)[KSTEPS][NTW], int k0) {
    const int klen = min(KC, kend - k0);
#pragma unroll
    for (int u = 0; u < KSTEPS; ++u)
#pragma unroll
      for (int n = 0; n < NTW; ++n)
        if (32 * u < klen) wf[u][n] = ldnt_bf16x8(wrow[n] + k0 + 32 * u);
  };

  f32x4 acc[MT][NTW];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](const bf16x8 (&wf)[KSTEPS][NTW], int buf, int k0) {
    const int klen = min(KC, kend - k0);
#pragma unroll
    for (int u = 0; u < KSTEPS; ++u) {
      if (32 * u >= klen) break;
      bf16x8 xf[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m)
        xf[m] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(&xs[buf][16 * m + r16][32 * u + 8 * g]));
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NTW; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xf[m], wf[u][n], acc[m][n], 0, 0, 0);
    }
  };

  if (nch > 0) {
    bf16x8 wa[KSTEPS][NTW], wb[KSTEPS][NTW];
    loadw(wa, kbeg);
    stage(0, kbeg);
    __syncthreads();
    for (int c = 0; c < nch; c += 2) {
      const int k0 = kbeg + c * KC;
      if (c + 1 < nch) {
        loadw(wb, k0 + KC);
        stage(1, k0 + KC);
      }
      compute(wa, 0, k0);
      __syncthreads();  // buffer 1 staged; buffer 0 free
      if (c + 1 < nch) {
        if (c + 2 < nch) {
          loadw(wa, k0 + 2 * KC);
          stage(0, k0 + 2 * KC);
        }
        compute(wb, 1, k0 + KC);
        __syncthreads();
      }
    }
  }

  // ---- epilogue: acc[m][n][r] = C[row 16m + 4g + r][col col0 + 16n + r16]
  const int rows = min(M, MP);
  if (S == 1) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < NTW; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * m + 4 * g + r, col = col0 + 16 * n + r16;
          if (row < rows && col < N) Y[(long)row * ldy + col] = f2bf(acc[m][n][r]);
        }
    return;
  }
  // split-K slab [split][tile] of NC columns x MP rows (column-major: a lane's 4 accumulator rows
  // are contiguous -> one 16-B write-through store), ticket, last arriver reduces with sc1 loads.
  const long slab_elems = (long)MP * NC;
  const __amdgpu_buffer_rsrc_t pr = make_rsrc(part, (unsigned)min((long)gridDim.x * gridDim.y * slab_elems * 4, 0x7fffffffL));
  const long my_slab = ((long)split * gridDim.x + tile) * slab_elems;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < NTW; ++n) {
      const int c = wave * 16 * NTW + 16 * n + r16;
      st_wt16(pr, (unsigned)((my_slab + (long)c * MP + 16 * m + 4 * g) * 4),
              make_float4(acc[m][n][0], acc[m][n][1], acc[m][n][2], acc[m][n][3]));
    }
  if (!ticket_last(&counters[tile], S, &s_last)) return;
  for (int e = tid * 4; e < NC * MP; e += 256 * 4) {
    const int c = e / MP, r0 = e % MP;
    if (r0 >= rows) continue;
    float4 v = {0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < S; ++sp) {
      const float4 q = ld_wt16(pr, (unsigned)(((((long)sp * gridDim.x + tile) * slab_elems) + e) * 4));
      v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
    }
    const int col = tile * NC + c;
    if (col >= N) continue;
    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (r0 + j < rows) Y[(long)(r0 + j) * ldy + col] = f2bf(vv[j]);
  }
}

template <int MT, int NTW, bool SW>
int launch(const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K, int splits, float* part,
           int* counters, hipStream_t st) {
  const int tiles = (N + 64 * NTW - 1) / (64 * NTW);
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + 31) & ~31;
  const int S = (K + kchunk - 1) / kchunk;
  hipLaunchKernelGGL((skinny_lds_kernel<MT, NTW, SW>), dim3(tiles, S), dim3(256), 0, st, (const u16*)X, ldx,
                     (const u16*)W, (u16*)Y, ldy, M, N, K, kchunk, part, counters);
  return (int)hipGetLastError();
}

template <int MT, bool SW>
int by_ntw(int ntw, const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K, int splits,
           float* part, int* counters, hipStream_t st) {
  switch (ntw) {
    case 1: return launch<MT, 1, SW>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
    case 2: return launch<MT, 2, SW>(X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
    default: return -10;
  }
}

template <bool SW>
int by_mt(int M, int ntw, const void* X, long ldx, const void* W, void* Y, long ldy, int N, int K, int splits,
          float* part, int* counters, hipStream_t st) {
  if (M <= 16) return by_ntw<1, SW>(ntw, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  if (M <= 32) return by_ntw<2, SW>(ntw, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  if (M <= 64) return by_ntw<4, SW>(ntw, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  if (M <= 128 && ntw == 1) return by_ntw<8, SW>(ntw, X, ldx, W, Y, ldy, M, N, K, splits, part, counters, st);
  return -11;
}
}  // namespace

// part: >= splits * ceil(N/(64 ntw)) * 64 ntw * 16 ceil(M/16) floats; counters >= ceil(N/(64 ntw)), zeroed.
extern "C" int dllm_skinny_lds_gemm(const void* X, long ldx, const void* W, void* Y, long ldy, int M, int N, int K,
                                    int ntw, int splits, int swiglu, float* part, int* counters, hipStream_t stream) {
  if (K % 32 != 0 || M <= 0 || M > 128 || splits < 1) return -1;
  if (splits > 1 && (!part || !counters)) return -2;
  return swiglu ? by_mt<true>(M, ntw, X, ldx, W, Y, ldy, N, K, splits, part, counters, stream)
                : by_mt<false>(M, ntw, X, ldx, W, Y, ldy, N, K, splits, part, counters, stream);
}
