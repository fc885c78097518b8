// A-direct decode-GEMM lab: Y[M, N] = X[M, K] . W[N, K]^T at the serving batch (M = 320-512).
//
// Round-4 probes (profiles/r4_decode_gemm_operands.md) found the shared ACTIVATION fill through
// the LDS-DMA ring to be as slow as the weight stream (~35-45 GB/s per CU each), and the two
// streams share one intake.  This kernel splits them over the two paths a CU has:
//   * W (read once per m-tile, shared by every wave of the workgroup) through an LDS-DMA ring
//     filled by NL dedicated loader waves (counted vmcnt, one raw barrier per 64-deep k-step);
//   * X straight into the VGPRs of the compute waves (global_load_dwordx4 from L2, PF k-steps
//     ahead), which are split over M so no two waves of a workgroup load the same activation row.
// Compute waves never issue LDS-DMA and loader waves never issue ordinary loads, so each wave's
// vmcnt counts exactly one stream (no compiler-inserted drains of the ring).
//
// Compared in the same process with the production tgemm (PLAIN epilogue), best plan per shape.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o expbin/adlab scripts/exp/adlab.hip
// Run:   ./adlab [M]   -> one JSON line per (shape, kernel, plan)
#include "../../csrc/kernels/tgemm.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include <math.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

namespace ad {
constexpr int BK = 64, ROWB = 128;

template <int N>
__device__ __forceinline__ void vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
template <int G, int MAXR>
__device__ __forceinline__ void wait_r(int r) {
  if constexpr (MAXR >= 6) { if (r >= 6) { vm<6 * G>(); return; } }
  if constexpr (MAXR >= 5) { if (r == 5) { vm<5 * G>(); return; } }
  if constexpr (MAXR >= 4) { if (r == 4) { vm<4 * G>(); return; } }
  if constexpr (MAXR >= 3) { if (r == 3) { vm<3 * G>(); return; } }
  if constexpr (MAXR >= 2) { if (r == 2) { vm<2 * G>(); return; } }
  if constexpr (MAXR >= 1) { if (r == 1) { vm<G>(); return; } }
  vm<0>();
}
__device__ __forceinline__ void bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// BM x BN output tile; NC compute waves each own BM/NC rows x all BN columns; NL loader waves;
// ST-slot W ring (BN rows x 128 B per slot); PF: k-steps of X held in registers ahead of use.
// ROT: rotated k start per tile.  Grid: mt * nt workgroups, XCD-aware order (the m-tiles of one
// n-tile on one XCD, so each XCD's L2 fetches a weight tile once).
template <int BM, int BN, int NC, int NL, int ST, int PF, bool ROT>
__global__ void __launch_bounds__(64 * (NC + NL)) ad_kernel(const u16* __restrict__ A, long lda,
                                                           const u16* __restrict__ W, u16* __restrict__ Y,
                                                           int M, int N, int K) {
  constexpr int WM = BM / NC, FM = WM / 16, FN = BN / 16;
  static_assert(WM % 16 == 0 && FM >= 1 && BN % 16 == 0, "wave tile");
  constexpr int SLOT = BN * ROWB;
  constexpr int PIECES = BN / 8;  // 1 KB glds pieces per slot
  static_assert(PIECES % NL == 0, "pieces per loader");
  constexpr int GL = PIECES / NL;
  __shared__ __attribute__((aligned(16))) unsigned char smem[ST * SLOT];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool loader = wid >= NC;
  const int mt = (M + BM - 1) / BM, nt = (N + BN - 1) / BN;
  const int nblk = mt * nt;
  int bid = blockIdx.x;
  {  // XCD-aware bijection: blocks b, b+8, b+16, ... (one XCD) get consecutive logical ids
    const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8, lin = bid / 8;
    bid = xcd * q8 + (xcd < r8 ? xcd : r8) + lin;
  }
  const int n_tile = bid / mt, m_tile = bid % mt;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int nk = K / BK;
  const int krot = ROT ? (int)((unsigned)(n_tile * 7 + m_tile * 3) % (unsigned)nk) : 0;
  auto kstep = [&](int t) { const int u = t + krot; return u >= nk ? u - nk : u; };

  if (loader) {
    const int lw = wid - NC, srow = lane >> 3, spos = lane & 7;
    const u16* src[GL];
    int off[GL];
#pragma unroll
    for (int j = 0; j < GL; ++j) {
      const int p = lw + NL * j, r = 8 * p + srow;
      src[j] = W + (long)min(n0 + r, N - 1) * K + 8 * (spos ^ ((r >> 1) & 7));
      off[j] = p * 1024;
    }
    auto issue = [&](int t) {
      unsigned char* base = smem + (t % ST) * SLOT;
      const int ko = kstep(t) * BK;
#pragma unroll
      for (int j = 0; j < GL; ++j)
        __builtin_amdgcn_global_load_lds((const void*)(src[j] + ko), (lds_void*)(base + off[j]), 16, 0, 0);
    };
#pragma unroll
    for (int t = 0; t < ST - 1; ++t)
      if (t < nk) issue(t);
    for (int t = 0; t < nk; ++t) {
      wait_r<GL, (ST - 2 < 6 ? ST - 2 : 6)>(min(ST - 2, nk - 1 - t));
      bar();
      if (t + ST - 1 < nk) issue(t + ST - 1);
    }
    return;
  }

  // ---- compute waves
  const int rbase = m0 + wid * WM + (lane & 15);
  const u16* arow[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) arow[i] = A + (long)min(rbase + 16 * i, M - 1) * lda + 8 * (lane >> 4);
  bf16x8 xa[PF][FM][2];
  auto loadx = [&](bf16x8 (&dst)[FM][2], int t) {
    const int ko = kstep(t) * BK;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) dst[i][h] = *reinterpret_cast<const bf16x8*>(arow[i] + ko + 32 * h);
  };
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (p < nk) loadx(xa[p], p);

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int t0 = 0; t0 < nk; t0 += PF) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int t = t0 + p;
      if (t < nk) {
        bar();  // slot t % ST landed (loaders waited), slot (t-1) % ST free for the refill
        const unsigned char* base = smem + (t % ST) * SLOT;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int c = 4 * h + (lane >> 4);
          bf16x8 bw[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int r = 16 * j + (lane & 15);
            bw[j] = *reinterpret_cast<const bf16x8*>(base + r * ROWB + ((c ^ ((r >> 1) & 7)) << 4));
          }
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[p][i][h], bw[j], acc[i][j], 0, 0, 0);
        }
        if (t + PF < nk) loadx(xa[p], t + PF);
      }
    }
  }
  // plain bf16 store: lane holds rows 4 (lane >> 4) + e, column lane & 15 of each fragment
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = m0 + wid * WM + 16 * i + 4 * (lane >> 4) + e;
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + 16 * j + (lane & 15);
        if (n < N) Y[(long)m * N + n] = f2bf(acc[i][j][e]);
      }
    }
}

__global__ void ref_kernel(const u16* A, long lda, const u16* W, float* Y, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(A[(long)m * lda + k]) * bf2f(W[(long)n * K + k]);
  Y[(long)m * N + n] = s;
}
}  // namespace ad

struct Var {
  const char* name;
  void (*launch)(const u16*, long, const u16*, u16*, int, int, int, hipStream_t);
  int bm, bn;
};

template <int BM, int BN, int NC, int NL, int ST, int PF, bool ROT>
void launch_ad(const u16* A, long lda, const u16* W, u16* Y, int M, int N, int K, hipStream_t s) {
  const int nb = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL((ad::ad_kernel<BM, BN, NC, NL, ST, PF, ROT>), dim3(nb), dim3(64 * (NC + NL)), 0, s, A, lda, W, Y, M,
                     N, K);
}

#define V(BM, BN, NC, NL, ST, PF, ROT) \
  Var{#BM "x" #BN " nc" #NC " nl" #NL " st" #ST " pf" #PF " rot" #ROT, launch_ad<BM, BN, NC, NL, ST, PF, ROT>, BM, BN}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 512;
  struct Shape { const char* name; int N, K; };
  const Shape shapes[] = {{"qkv", 2560, 2048}, {"wo", 2048, 2048}, {"gateup", 11264, 2048}, {"down", 2048, 5632}};
  const Var vars[] = {
      V(64, 64, 4, 2, 6, 2, false),  V(64, 64, 4, 2, 6, 3, false),  V(64, 64, 4, 4, 8, 2, false),
      V(64, 64, 4, 2, 6, 2, true),   V(128, 64, 8, 2, 6, 2, false), V(64, 128, 4, 4, 6, 2, false),
      V(64, 128, 4, 2, 6, 2, false), V(128, 128, 8, 4, 6, 2, false), V(32, 64, 2, 2, 6, 2, false),
      V(64, 32, 4, 2, 8, 2, false),  V(128, 32, 8, 2, 8, 2, false), V(64, 64, 2, 2, 6, 2, false),
  };
  // production tgemm plans (PLAIN) for the comparison column
  struct TPlan { int bm, bn, st, ks, nw, nl; };
  const TPlan tplans[] = {{64, 64, 3, 2, 4, 0}, {64, 128, 3, 2, 8, 0}, {64, 64, 4, 1, 4, 8}, {128, 64, 4, 1, 4, 8},
                          {256, 128, 3, 1, 8, 8}};
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  const int Kmax = 5632, Nmax = 11264;
  u16 *A, *Y;
  float *Yr, *part;
  int* cnt;
  CHECK(hipMalloc(&A, (long)M * Kmax * 2));
  CHECK(hipMalloc(&Y, (long)M * Nmax * 2));
  CHECK(hipMalloc(&Yr, (long)M * Nmax * 4));
  CHECK(hipMalloc(&part, (64L << 20) * 4));
  CHECK(hipMalloc(&cnt, 1 << 20));
  CHECK(hipMemset(cnt, 0, 1 << 20));
  srand(5);
  {
    std::vector<u16> a((long)M * Kmax);
    for (auto& x : a) { float f = rand() / (float)RAND_MAX - 0.5f; uint32_t u; memcpy(&u, &f, 4); x = u >> 16; }
    CHECK(hipMemcpy(A, a.data(), a.size() * 2, hipMemcpyHostToDevice));
  }
  std::vector<float> yr, yb;
  std::vector<u16> yh;
  for (const Shape& sh : shapes) {
    const long wel = (long)sh.N * sh.K;
    const int copies = (int)std::max(2L, std::min(48L, (640L << 20) / (wel * 2)));
    const int nlaunch = std::max(copies, 48);
    std::vector<u16*> ws(copies);
    std::vector<u16> hw(wel);
    for (auto& x : hw) { float f = (rand() / (float)RAND_MAX - 0.5f) * 0.05f; uint32_t u; memcpy(&u, &f, 4); x = u >> 16; }
    for (auto& w : ws) {
      CHECK(hipMalloc(&w, wel * 2));
      CHECK(hipMemcpy(w, hw.data(), wel * 2, hipMemcpyHostToDevice));
    }
    hipLaunchKernelGGL(ad::ref_kernel, dim3((sh.N + 255) / 256, M), dim3(256), 0, s, A, (long)sh.K, ws[0], Yr, M, sh.N, sh.K);
    CHECK(hipStreamSynchronize(s));
    yr.resize((long)M * sh.N);
    CHECK(hipMemcpy(yr.data(), Yr, yr.size() * 4, hipMemcpyDeviceToHost));
    auto check = [&]() -> double {
      yh.resize((long)M * sh.N);
      CHECK(hipMemcpy(yh.data(), Y, yh.size() * 2, hipMemcpyDeviceToHost));
      double err = 0;
      for (long i = 0; i < (long)yh.size(); ++i) {
        uint32_t u = (uint32_t)yh[i] << 16; float f; memcpy(&f, &u, 4);
        err = std::max(err, (double)fabsf(f - yr[i]));
      }
      return err;
    };
    auto timeit = [&](auto&& fn) -> double {
      hipGraph_t g;
      hipGraphExec_t ge;
      CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int i = 0; i < nlaunch; ++i) fn(ws[i % copies]);
      CHECK(hipStreamEndCapture(s, &g));
      CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CHECK(hipGraphLaunch(ge, s));
      CHECK(hipStreamSynchronize(s));
      hipEvent_t e0, e1;
      CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
      const int reps = 6;
      CHECK(hipEventRecord(e0, s));
      for (int r = 0; r < reps; ++r) CHECK(hipGraphLaunch(ge, s));
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(g));
      return ms * 1000.0 / (reps * nlaunch);
    };
    for (const TPlan& p : tplans) {
      dllm::GemmArgs a{};
      a.A = A; a.lda = sh.K; a.M = M; a.N = sh.N; a.K = sh.K; a.splits = 1; a.kchunk = sh.K;
      a.part = part; a.counters = cnt; a.W = ws[0]; a.Y = Y; a.ldy = sh.N;
      if (dllm_tgemm(&a, p.bm, p.bn, p.st, p.ks, p.nw, 1, dllm::EPI_PLAIN, s, p.nl) != 0) continue;
      CHECK(hipStreamSynchronize(s));
      const double err = check();
      const double us = timeit([&](u16* w) { a.W = w; dllm_tgemm(&a, p.bm, p.bn, p.st, p.ks, p.nw, 1, dllm::EPI_PLAIN, s, p.nl); });
      printf("{\"M\": %d, \"shape\": \"%s\", \"kernel\": \"tgemm\", \"plan\": \"%dx%d st%d ks%d nw%d nl%d\", \"us\": %.2f, \"TFs\": %.0f, \"err\": %.4f}\n",
             M, sh.name, p.bm, p.bn, p.st, p.ks, p.nw, p.nl, us, 2.0 * M * sh.N * sh.K / us / 1e6, err);
      fflush(stdout);
    }
    for (const Var& v : vars) {
      if (sh.N % v.bn != 0) continue;
      CHECK(hipMemset(Y, 0, (long)M * sh.N * 2));
      v.launch(A, sh.K, ws[0], Y, M, sh.N, sh.K, s);
      CHECK(hipStreamSynchronize(s));
      const double err = check();
      const double us = timeit([&](u16* w) { v.launch(A, sh.K, w, Y, M, sh.N, sh.K, s); });
      printf("{\"M\": %d, \"shape\": \"%s\", \"kernel\": \"adirect\", \"plan\": \"%s\", \"wgs\": %d, \"us\": %.2f, \"TFs\": %.0f, \"err\": %.4f}\n",
             M, sh.name, v.name, ((M + v.bm - 1) / v.bm) * (sh.N / v.bn), us, 2.0 * M * sh.N * sh.K / us / 1e6, err);
      fflush(stdout);
    }
    for (auto& w : ws) CHECK(hipFree(w));
  }
  return 0;
}
