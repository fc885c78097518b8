// Mixture-of-experts FFN for Mixtral-style top-k routing — graph-capturable (no host sync).
//
//   moe_route   : one workgroup turns the top-k expert ids [T*k] into an expert-sorted pair list
//                 (perm) and a tile list (expert, first row, rows) of MT-row tiles; the tile count
//                 lives on the device, so a captured decode graph handles any routing.
//   moe_gemm13  : grouped GEMM over the tile list: rows gathered through perm straight from the
//                 token activations (no materialised permuted copy), gate and up columns of the
//                 expert's fused w13 in the same wave, SiLU(gate)*up in the epilogue -> act.
//   moe_gemm2   : grouped down projection act . w2_e^T, scaled by the pair's gate weight and
//                 written to the pair's own slot (token-major, [T*k, H] f32)
//   moe_combine : out[t] = sum_j y[t*k + j] in fixed order -> deterministic, no atomics.
// MFMA: v_mfma_f32_16x16x32_bf16; A = 16 gathered rows x 32 k (row lane&15, k 8(lane>>4)+j),
// B = 32 k x 16 weight rows (same pattern on the [N, K] weight), C row (lane>>4)*4+r, col lane&15.
// Tiles are MT = 32 rows (two MFMA row groups share every weight load); blocks past the device
// tile count exit immediately.  Weights stream with 4 k-steps of loads in flight per wave.
//
// moe_ffn_tg (the default on GPU): the same routing with BM-row tiles, then BOTH expert GEMMs on
// the LDS-tiled MFMA GEMM of tgemm.hip in grouped mode — global_load_lds ring, XOR-swizzled LDS,
// rows of the first GEMM gathered through perm by the staging addresses, the expert's weight
// slice picked per row tile, SwiGLU in the epilogue over gate/up rows interleaved in 16-row
// groups (models.llama.interleave_w13) — and a combine that applies the gate weights while
// summing each token's k expert rows (inverse permutation, fixed order, no atomics).
#include "common.h"
#include "tgemm_args.h"

extern "C" int dllm_tgemm(const void* args, int bm, int bn, int stages, int ks, int nw, int wk, int epi,
                          hipStream_t stream, int nl);

namespace {
constexpr int MT = 32;

__global__ void __launch_bounds__(1024) moe_route_kernel(const int* __restrict__ ids, int P, int E, int max_tiles,
                                                         int* __restrict__ perm, int* __restrict__ tile_e,
                                                         int* __restrict__ tile_r0, int* __restrict__ tile_n,
                                                         int* __restrict__ n_tiles, int mt = MT,
                                                         int* __restrict__ inv = nullptr) {
  // Pairs are placed in a stable order (pair index ascending within each expert): per chunk of
  // blockDim pairs, a pair's slot = expert base + pairs of its expert in earlier chunks + in earlier
  // waves of this chunk + lower lanes of its wave (ballot ranks), so the layout never depends on
  // atomic arrival order.
  __shared__ int cnt[64], off[65], cur[64], wcnt[16][64];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nwv = blockDim.x >> 6;
  if (tid < 64) { cnt[tid] = 0; cur[tid] = 0; }
  __syncthreads();
  for (int p = tid; p < P; p += blockDim.x) atomicAdd(&cnt[min(max(ids[p], 0), E - 1)], 1);  // order-free sum
  __syncthreads();
  if (tid == 0) {
    off[0] = 0;
    for (int e = 0; e < E; ++e) off[e + 1] = off[e] + cnt[e];
    int nt = 0;
    for (int e = 0; e < E; ++e)
      for (int r = 0; r < cnt[e] && nt < max_tiles; r += mt, ++nt) {
        tile_e[nt] = e;
        tile_r0[nt] = off[e] + r;
        tile_n[nt] = min(mt, cnt[e] - r);
      }
    *n_tiles = nt;
  }
  __syncthreads();
  for (int base = 0; base < P; base += blockDim.x) {  // uniform trip count: every wave ballots
    const int p = base + tid;
    const int e = p < P ? min(max(ids[p], 0), E - 1) : -1;
    int rank = 0;
    for (int x = 0; x < E; ++x) {
      const unsigned long long m = __ballot(e == x);
      if (e == x) rank = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) wcnt[wv][x] = __popcll(m);
    }
    __syncthreads();
    if (e >= 0) {
      int pos = off[e] + cur[e] + rank;
      for (int v = 0; v < wv; ++v) pos += wcnt[v][e];
      perm[pos] = p;
      if (inv != nullptr) inv[p] = pos;
    }
    __syncthreads();
    if (tid < E) {
      int s = 0;
      for (int v = 0; v < nwv; ++v) s += wcnt[v][tid];
      cur[tid] += s;
    }
    __syncthreads();
  }
}

// out[t] = sum_j wts[t k + j] * y[inv[t k + j]]  (y: expert outputs in expert-sorted row order)
__global__ void moe_combine_perm_kernel(const u16* __restrict__ y, const int* __restrict__ inv,
                                        const float* __restrict__ wts, int k, int H, long T, u16* __restrict__ out) {
  const long n8 = T * (H / 8);
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n8; v += (long)gridDim.x * blockDim.x) {
    const long t = v / (H / 8);
    const int h = (int)(v % (H / 8)) * 8;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const long p = t * k + j;
      float f[8];
      unpack8(ld16(y + (long)inv[p] * H + h), f);
      const float w = wts[p];
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += w * f[q];
    }
    st16(out + t * (long)H + h, pack8(s));
  }
}

__device__ __forceinline__ bf16x8 ld_or0(const u16* p, bool ok) {
  return __builtin_bit_cast(bf16x8, ok ? ld16(p) : make_uint4(0, 0, 0, 0));
}

// act[row, c] = silu(x_row . wg_c) * (x_row . wu_c); block = 4 waves x 16 columns, MT rows.
__global__ void __launch_bounds__(256) moe_gemm13_kernel(const u16* __restrict__ x, long x_stride,
                                                         const int* __restrict__ perm, int k,
                                                         const int* __restrict__ tile_e,
                                                         const int* __restrict__ tile_r0,
                                                         const int* __restrict__ tile_n,
                                                         const int* __restrict__ n_tiles,
                                                         const u16* __restrict__ w13, u16* __restrict__ act, int I,
                                                         int H) {
  const int tile = blockIdx.x;
  if (tile >= *n_tiles) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col0 = blockIdx.y * 64 + wave * 16;
  if (col0 >= I) return;  // whole wave; the kernel has no block-level barrier
  const int e = tile_e[tile], r0 = tile_r0[tile], nrows = tile_n[tile];
  const int rl = lane & 15, kq = 8 * (lane >> 4);
  const u16* arow[2];
  bool aok[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int row = 16 * g + rl;
    aok[g] = row < nrows;
    const int pair = aok[g] ? perm[r0 + row] : 0;
    arow[g] = x + (long)(pair / k) * x_stride + kq;
  }
  const int n = col0 + rl;
  const bool nok = n < I;
  const u16* wg = w13 + ((long)e * 2 * I + (nok ? n : 0)) * H + kq;
  const u16* wu = wg + (long)I * H;
  f32x4 ag[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  f32x4 au[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  int kk = 0;
  for (; kk + 128 <= H; kk += 128) {
    bf16x8 a[4][2], bg[4], bu[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bg[s] = ld_or0(wg + kk + 32 * s, nok);
      bu[s] = ld_or0(wu + kk + 32 * s, nok);
#pragma unroll
      for (int g = 0; g < 2; ++g) a[s][g] = ld_or0(arow[g] + kk + 32 * s, aok[g]);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        ag[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][g], bg[s], ag[g], 0, 0, 0);
        au[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][g], bu[s], au[g], 0, 0, 0);
      }
  }
  for (; kk < H; kk += 32) {
    const bf16x8 bgs = ld_or0(wg + kk, nok), bus = ld_or0(wu + kk, nok);
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const bf16x8 as = ld_or0(arow[g] + kk, aok[g]);
      ag[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as, bgs, ag[g], 0, 0, 0);
      au[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as, bus, au[g], 0, 0, 0);
    }
  }
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * g + (lane >> 4) * 4 + r;
      if (row < nrows && nok) {
        const float gv = ag[g][r];
        act[(long)(r0 + row) * I + n] = f2bf(gv / (1.f + __expf(-gv)) * au[g][r]);
      }
    }
}

// y[pair, c] = gate_w[pair] * (act_row . w2_e[c]); block = 4 waves x 32 columns, MT rows.
__global__ void __launch_bounds__(256) moe_gemm2_kernel(const u16* __restrict__ act, const int* __restrict__ perm,
                                                        const float* __restrict__ wts,
                                                        const int* __restrict__ tile_e,
                                                        const int* __restrict__ tile_r0,
                                                        const int* __restrict__ tile_n,
                                                        const int* __restrict__ n_tiles, const u16* __restrict__ w2,
                                                        float* __restrict__ y, int I, int H) {
  const int tile = blockIdx.x;
  if (tile >= *n_tiles) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col0 = blockIdx.y * 128 + wave * 32;
  if (col0 >= H) return;
  const int e = tile_e[tile], r0 = tile_r0[tile], nrows = tile_n[tile];
  const int rl = lane & 15, kq = 8 * (lane >> 4);
  const u16* arow[2];
  bool aok[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int row = 16 * g + rl;
    aok[g] = row < nrows;
    arow[g] = act + (long)(r0 + (aok[g] ? row : 0)) * I + kq;
  }
  const u16* wb[2];
  bool nok[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int n = col0 + 16 * c + rl;
    nok[c] = n < H;
    wb[c] = w2 + ((long)e * H + (nok[c] ? n : 0)) * I + kq;
  }
  f32x4 acc[2][2] = {};
  int kk = 0;
  for (; kk + 128 <= I; kk += 128) {
    bf16x8 a[4][2], b[4][2];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        b[s][g] = ld_or0(wb[g] + kk + 32 * s, nok[g]);
        a[s][g] = ld_or0(arow[g] + kk + 32 * s, aok[g]);
      }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          acc[g][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][g], b[s][c], acc[g][c], 0, 0, 0);
  }
  for (; kk < I; kk += 32) {
    bf16x8 a[2], b[2];
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      a[g] = ld_or0(arow[g] + kk, aok[g]);
      b[g] = ld_or0(wb[g] + kk, nok[g]);
    }
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        acc[g][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[g], b[c], acc[g][c], 0, 0, 0);
  }
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * g + (lane >> 4) * 4 + r;
      if (row >= nrows) continue;
      const int pair = perm[r0 + row];
      const float sc = wts[pair];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int n = col0 + 16 * c + rl;
        if (nok[c]) y[(long)pair * H + n] = sc * acc[g][c][r];
      }
    }
}

__global__ void moe_combine_kernel(const float* __restrict__ y, int k, int H, long T, u16* __restrict__ out) {
  const long n4 = T * (H / 4);
  for (long v = blockIdx.x * (long)blockDim.x + threadIdx.x; v < n4; v += (long)gridDim.x * blockDim.x) {
    const long t = v / (H / 4);
    const int h = (int)(v % (H / 4)) * 4;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const float4 q = *reinterpret_cast<const float4*>(y + ((t * k + j) * (long)H + h));
      s[0] += q.x; s[1] += q.y; s[2] += q.z; s[3] += q.w;
    }
    u16* o = out + t * (long)H + h;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = f2bf(s[j]);
  }
}
}  // namespace

extern "C" int dllm_moe_max_tiles(int P, int E) { return (P + MT - 1) / MT + E; }

extern "C" int dllm_moe_ffn(const void* x, long x_stride, long T, int H, const int* ids, const float* wts, int k,
                            int E, const void* w13, const void* w2, int I, int* perm, int* tiles /*4 x max_tiles*/,
                            void* act, float* y, void* out, hipStream_t stream) {
  if (E < 1 || E > 64 || k < 1 || H % 32 != 0 || I % 32 != 0 || H % 4 != 0) return -1;
  if (T == 0) return 0;
  const int P = (int)(T * k);
  const int max_tiles = (P + MT - 1) / MT + E;
  int *te = tiles, *tr = tiles + max_tiles, *tn = tiles + 2 * max_tiles, *nt = tiles + 3 * max_tiles;
  hipLaunchKernelGGL(moe_route_kernel, dim3(1), dim3(1024), 0, stream, ids, P, E, max_tiles, perm, te, tr, tn, nt);
  hipLaunchKernelGGL(moe_gemm13_kernel, dim3(max_tiles, (I + 63) / 64), dim3(256), 0, stream, (const u16*)x,
                     x_stride, perm, k, te, tr, tn, nt, (const u16*)w13, (u16*)act, I, H);
  hipLaunchKernelGGL(moe_gemm2_kernel, dim3(max_tiles, (H + 127) / 128), dim3(256), 0, stream, (const u16*)act, perm,
                     wts, te, tr, tn, nt, (const u16*)w2, y, I, H);
  long n4 = T * (H / 4);
  long g = (n4 + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(moe_combine_kernel, dim3((int)g), dim3(256), 0, stream, y, k, H, T, (u16*)out);
  return (int)hipGetLastError();
}

// Tile-list size for BM-row tiles: every expert may leave one partial tile.
extern "C" int dllm_moe_max_tiles_bm(int P, int E, int bm) { return (P + bm - 1) / bm + E; }

// plans: {bm, bn13, stages13, ks13, nw13, bn2, stages2, ks2, nw2}; w13 interleaved [E, 2I, H]
// (16 gate rows, 16 up rows, ...), w2 [E, H, I]; scratch: perm/inv [P], tiles [4 * max_tiles + 1],
// act [P, I], y [P, H] (bf16).
extern "C" int dllm_moe_ffn_tg(const void* x, long x_stride, long T, int H, const int* ids, const float* wts, int k,
                               int E, const void* w13, const void* w2, int I, int* perm, int* inv, int* tiles,
                               void* act, void* y, void* out, const int* plan, hipStream_t stream) {
  if (E < 1 || E > 64 || k < 1 || H % 64 != 0 || I % 64 != 0 || x_stride % 8) return -1;
  if (T == 0) return 0;
  const int bm = plan[0];
  const int P = (int)(T * k);
  const int max_tiles = (P + bm - 1) / bm + E;
  int *te = tiles, *tr = tiles + max_tiles, *tn = tiles + 2 * max_tiles, *nt = tiles + 3 * max_tiles;
  hipLaunchKernelGGL(moe_route_kernel, dim3(1), dim3(1024), 0, stream, ids, P, E, max_tiles, perm, te, tr, tn, nt, bm,
                     inv);
  dllm::GemmArgs g{};
  g.A = (const uint16_t*)x; g.lda = x_stride; g.W = (const uint16_t*)w13; g.Y = (uint16_t*)act; g.ldy = I;
  g.M = max_tiles * bm; g.N = 2 * I; g.K = H; g.kchunk = H; g.splits = 1;
  g.g_tiles = tiles; g.g_max = max_tiles; g.g_perm = perm; g.g_k = k; g.g_wstride = 2L * I * H;
  int rc = dllm_tgemm(&g, bm, plan[1], plan[2], plan[3], plan[4], 1, dllm::EPI_SWIGLU, stream, 0);
  if (rc) return 1000 + rc;
  dllm::GemmArgs d{};
  d.A = (const uint16_t*)act; d.lda = I; d.W = (const uint16_t*)w2; d.Y = (uint16_t*)y; d.ldy = H;
  d.M = max_tiles * bm; d.N = H; d.K = I; d.kchunk = I; d.splits = 1;
  d.g_tiles = tiles; d.g_max = max_tiles; d.g_perm = nullptr; d.g_k = 1; d.g_wstride = (long)H * I;
  rc = dllm_tgemm(&d, bm, plan[5], plan[6], plan[7], plan[8], 1, dllm::EPI_PLAIN, stream, 0);
  if (rc) return 2000 + rc;
  long n8 = T * (H / 8);
  long gr = (n8 + 255) / 256;
  if (gr > 4096) gr = 4096;
  hipLaunchKernelGGL(moe_combine_perm_kernel, dim3((int)gr), dim3(256), 0, stream, (const u16*)y, inv, wts, k, H, T,
                     (u16*)out);
  return (int)hipGetLastError();
}
