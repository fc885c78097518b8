// Experiment: what read bandwidth does the paged-KV access pattern of decode attention allow?
// (TinyLlama decode shape: nkv = 4, d = 64, 16-token blocks, random block placement.)
// Kernels read the same bytes as decode attention and fold them into a checksum (no softmax/MFMA):
//   seq      : plain grid-stride streaming read of the whole K and V arrays (practical ceiling)
//   attnlike : one workgroup (8 waves) per (sequence, kv head), attention.hip's lane pattern
//              (K: 16 rows x 64 B half-lines per instruction; V: 8-B per lane)
//   fullline : same work split, lane-linear 16-B loads (each instruction = 8 whole 128-B lines)
//   allheads : one workgroup per sequence; wave w takes head w % nkv and every (8/nkv)-th chunk:
//              the 8 KB (all heads) of each block are read together
//   waveunit : every wave is an independent worker over (sequence, head, split) units, CH chunks
//              of loads in flight per wave, no barriers
// Build: hipcc --offload-arch=gfx950 -O3 -o kvread scripts/exp/kvread.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <random>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int BS = 16, D = 64;

__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

__global__ void k_seq(const uint4* __restrict__ a, long n16, uint32_t* out) {
  uint32_t acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n16; i += (long)gridDim.x * blockDim.x) acc ^= fold(a[i]);
  if (acc == 0x12345678u) out[0] = acc;
}

// NT: non-temporal loads (each K/V byte is read once per decode step by one workgroup)
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
template <typename T, bool NT>
__device__ __forceinline__ T ldk(const T* p) {
  if constexpr (NT) {
    if constexpr (sizeof(T) == 16) return __builtin_bit_cast(T, __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(p)));
    else return __builtin_bit_cast(T, __builtin_nontemporal_load(reinterpret_cast<const u32x2v*>(p)));
  } else {
    return *p;
  }
}

// head block = 16 keys x 64 dims bf16 = 2 KB; K [blocks][nkv][16][64], V [blocks][nkv][64][16]
template <bool NT = false>
__global__ void __launch_bounds__(512) k_attnlike(const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
                                                  const int* __restrict__ bt, int nb, int nkv, uint32_t* out) {
  const int seq = blockIdx.x / nkv, h = blockIdx.x % nkv;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, rl = lane & 15;
  uint32_t acc = 0;
  for (int c = wave; c < nb / 2; c += 8) {
    const int b0 = bt[seq * nb + 2 * c], b1 = bt[seq * nb + 2 * c + 1];
    const uint16_t* k0 = kc + ((long)b0 * nkv + h) * BS * D + rl * D + 8 * g;
    const uint16_t* k1 = kc + ((long)b1 * nkv + h) * BS * D + rl * D + 8 * g;
    const uint16_t* v0 = vc + ((long)b0 * nkv + h) * BS * D + rl * BS + 4 * g;
    const uint16_t* v1 = vc + ((long)b1 * nkv + h) * BS * D + rl * BS + 4 * g;
    uint4 kr[4];
    uint2 vr[8];
    kr[0] = ldk<uint4, NT>((const uint4*)(k0)); kr[1] = ldk<uint4, NT>((const uint4*)(k0 + 32));
    kr[2] = ldk<uint4, NT>((const uint4*)(k1)); kr[3] = ldk<uint4, NT>((const uint4*)(k1 + 32));
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      vr[n] = ldk<uint2, NT>((const uint2*)(v0 + 16 * n * BS));
      vr[4 + n] = ldk<uint2, NT>((const uint2*)(v1 + 16 * n * BS));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) acc ^= fold(kr[i]);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= vr[i].x ^ vr[i].y;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(512) k_fullline(const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
                                                  const int* __restrict__ bt, int nb, int nkv, uint32_t* out) {
  const int seq = blockIdx.x / nkv, h = blockIdx.x % nkv;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t acc = 0;
  for (int c = wave; c < nb / 2; c += 8) {
    const int b0 = bt[seq * nb + 2 * c], b1 = bt[seq * nb + 2 * c + 1];
    const uint4* k0 = (const uint4*)(kc + ((long)b0 * nkv + h) * BS * D);
    const uint4* k1 = (const uint4*)(kc + ((long)b1 * nkv + h) * BS * D);
    const uint4* v0 = (const uint4*)(vc + ((long)b0 * nkv + h) * BS * D);
    const uint4* v1 = (const uint4*)(vc + ((long)b1 * nkv + h) * BS * D);
    uint4 r[8] = {k0[lane], k0[64 + lane], k1[lane], k1[64 + lane], v0[lane], v0[64 + lane], v1[lane], v1[64 + lane]};
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= fold(r[i]);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(512) k_allheads(const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
                                                  const int* __restrict__ bt, int nb, int nkv, uint32_t* out) {
  const int seq = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = wave % nkv, par = wave / nkv, npar = 8 / nkv;
  uint32_t acc = 0;
  for (int c = par; c < nb / 2; c += npar) {
    const int b0 = bt[seq * nb + 2 * c], b1 = bt[seq * nb + 2 * c + 1];
    const uint4* k0 = (const uint4*)(kc + ((long)b0 * nkv + h) * BS * D);
    const uint4* k1 = (const uint4*)(kc + ((long)b1 * nkv + h) * BS * D);
    const uint4* v0 = (const uint4*)(vc + ((long)b0 * nkv + h) * BS * D);
    const uint4* v1 = (const uint4*)(vc + ((long)b1 * nkv + h) * BS * D);
    uint4 r[8] = {k0[lane], k0[64 + lane], k1[lane], k1[64 + lane], v0[lane], v0[64 + lane], v1[lane], v1[64 + lane]};
#pragma unroll
    for (int i = 0; i < 8; ++i) acc ^= fold(r[i]);
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// wave-independent units: unit u = (seq, head, split of `ns`); CH 32-key chunks loaded per trip
template <int CH>
__global__ void __launch_bounds__(256) k_waveunit(const uint16_t* __restrict__ kc, const uint16_t* __restrict__ vc,
                                                  const int* __restrict__ bt, int nb, int nkv, int ns, int nunits,
                                                  uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), nw = gridDim.x * (blockDim.x >> 6);
  uint32_t acc = 0;
  const int cps = (nb / 2 + ns - 1) / ns;  // chunks per split
  for (int u = wid; u < nunits; u += nw) {
    const int seq = u / (nkv * ns), h = (u / ns) % nkv, sp = u % ns;
    const int c0 = sp * cps, c1 = min(nb / 2, c0 + cps);
    for (int c = c0; c < c1; c += CH) {
      uint4 r[CH][8];
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int cc = min(c + j, c1 - 1);
        const int b0 = bt[seq * nb + 2 * cc], b1 = bt[seq * nb + 2 * cc + 1];
        const uint4* k0 = (const uint4*)(kc + ((long)b0 * nkv + h) * BS * D);
        const uint4* k1 = (const uint4*)(kc + ((long)b1 * nkv + h) * BS * D);
        const uint4* v0 = (const uint4*)(vc + ((long)b0 * nkv + h) * BS * D);
        const uint4* v1 = (const uint4*)(vc + ((long)b1 * nkv + h) * BS * D);
        r[j][0] = k0[lane]; r[j][1] = k0[64 + lane]; r[j][2] = k1[lane]; r[j][3] = k1[64 + lane];
        r[j][4] = v0[lane]; r[j][5] = v0[64 + lane]; r[j][6] = v1[lane]; r[j][7] = v1[64 + lane];
      }
#pragma unroll
      for (int j = 0; j < CH; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc ^= fold(r[j][i]);
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
float timeit(F f, int iters = 20) {
  for (int i = 0; i < 3; ++i) f();
  CHECK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 512, C = argc > 2 ? atoi(argv[2]) : 2048, nkv = 4;
  const int nb = C / BS;
  const long NB = (long)B * nb + 8;
  const long elems = NB * nkv * BS * D;
  uint16_t *kc, *vc;
  int* bt;
  uint32_t* out;
  CHECK(hipMalloc(&kc, elems * 2)); CHECK(hipMalloc(&vc, elems * 2));
  CHECK(hipMemset(kc, 1, elems * 2)); CHECK(hipMemset(vc, 2, elems * 2));
  CHECK(hipMalloc(&bt, (long)B * nb * 4)); CHECK(hipMalloc(&out, 64));
  std::vector<int> perm(NB - 8);
  for (long i = 0; i < NB - 8; ++i) perm[i] = (int)i;
  // placement: 0 every sequence's blocks consecutive, 1 random blocks, 2 runs of 64 consecutive
  // blocks at random places (the block manager's segment placement)
  const int shuffled = argc > 3 ? atoi(argv[3]) : 1;
  if (shuffled == 1) std::shuffle(perm.begin(), perm.end(), std::mt19937(1));
  if (shuffled == 2) {
    const long nseg = (NB - 8) / 64;
    std::vector<long> segs(nseg);
    for (long i = 0; i < nseg; ++i) segs[i] = i;
    std::shuffle(segs.begin(), segs.end(), std::mt19937(1));
    for (long i = 0; i < nseg * 64; ++i) perm[i] = (int)(segs[i / 64] * 64 + i % 64);
  }
  CHECK(hipMemcpy(bt, perm.data(), (long)B * nb * 4, hipMemcpyHostToDevice));
  const double bytes = (double)B * nb * nkv * BS * D * 2 * 2;
  auto rep = [&](const char* name, float ms) {
    printf("{\"exp\": \"kvread\", \"kernel\": \"%s\", \"B\": %d, \"C\": %d, \"shuffled\": %d, \"us\": %.1f, \"TBps\": %.3f}\n",
           name, B, C, (int)shuffled, ms * 1000, bytes / (ms * 1e-3) / 1e12);
  };
  {
    const long n16 = elems * 2 / 16;
    float ms = timeit([&] {
      hipLaunchKernelGGL(k_seq, dim3(4096), dim3(256), 0, 0, (const uint4*)kc, n16, out);
      hipLaunchKernelGGL(k_seq, dim3(4096), dim3(256), 0, 0, (const uint4*)vc, n16, out);
    });
    printf("{\"exp\": \"kvread\", \"kernel\": \"seq\", \"bytes\": %.0f, \"us\": %.1f, \"TBps\": %.3f}\n", (double)elems * 4,
           ms * 1000, elems * 4.0 / (ms * 1e-3) / 1e12);
  }
  rep("attnlike", timeit([&] { hipLaunchKernelGGL(k_attnlike<false>, dim3(B * nkv), dim3(512), 0, 0, kc, vc, bt, nb, nkv, out); }));
  rep("attnlike_nt", timeit([&] { hipLaunchKernelGGL(k_attnlike<true>, dim3(B * nkv), dim3(512), 0, 0, kc, vc, bt, nb, nkv, out); }));
  if (argc > 4) return 0;   // attnlike rows only
  rep("fullline", timeit([&] { hipLaunchKernelGGL(k_fullline, dim3(B * nkv), dim3(512), 0, 0, kc, vc, bt, nb, nkv, out); }));
  rep("allheads", timeit([&] { hipLaunchKernelGGL(k_allheads, dim3(B), dim3(512), 0, 0, kc, vc, bt, nb, nkv, out); }));
  for (int ns : {1, 2, 4}) {
    const int nunits = B * nkv * ns;
    for (int grid : {512, 1024, 2048}) {
      char name[64];
      snprintf(name, sizeof name, "waveunit_ch1_ns%d_g%d", ns, grid);
      rep(name, timeit([&] { hipLaunchKernelGGL(k_waveunit<1>, dim3(grid), dim3(256), 0, 0, kc, vc, bt, nb, nkv, ns, nunits, out); }));
      snprintf(name, sizeof name, "waveunit_ch2_ns%d_g%d", ns, grid);
      rep(name, timeit([&] { hipLaunchKernelGGL(k_waveunit<2>, dim3(grid), dim3(256), 0, 0, kc, vc, bt, nb, nkv, ns, nunits, out); }));
    }
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
