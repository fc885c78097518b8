// Experiment: how fast can ONE launch stream a decode weight matrix (8-235 MB, read once, no math)?
// The round-2 readfloor.hip kept one 16-B load in flight per thread; this probe keeps U loads in
// flight per lane and compares the three ways a GEMV can take its weights in:
//   vgpr    : U x global_load_dwordx4 to VGPRs per trip (default cache policy)
//   vgpr_nt : the same with the nontemporal bit (what gemv.hip uses)
//   lds_nt  : U x global_load_lds_dwordx4 (LDS-DMA, nt) into a per-wave LDS ring, vmcnt-counted
// Rows: (MB, grid, waves per WG, U) -> us per launch (hipGraph of rotated copies, so every launch
// reads HBM) and TB/s.  The decode GEMV at batch <= 8 cannot beat the best row.
// Build: hipcc --offload-arch=gfx950 -O3 -o labbin2/streamfloor scripts/exp/streamfloor.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

// Each wave streams contiguous 1 KB pieces: piece p = (wave_global + i * total_waves) for i < ...
template <int U, int MODE>
__global__ void k_stream(const uint4* __restrict__ a, long n_pieces, unsigned* out) {
  extern __shared__ uint4 ring[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const long wg = (long)blockIdx.x * nw + wave, tw = (long)gridDim.x * nw;
  unsigned acc = 0;
  for (long p0 = wg; p0 < n_pieces; p0 += tw * U) {
    if constexpr (MODE == 2) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long p = p0 + u * tw;
        if (p < n_pieces)
          __builtin_amdgcn_global_load_lds((const void*)(a + p * 64 + lane),
                                           (lds_void*)(ring + (wave * U + u) * 64), 16, 0, 2);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      acc ^= ring[(wave * U) * 64 + lane].x;
    } else {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long p = p0 + u * tw;
        if (p < n_pieces) {
          if constexpr (MODE == 1)
            v[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a + p * 64 + lane)));
          else
            v[u] = a[p * 64 + lane];
        } else {
          v[u] = make_uint4(0, 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int U, int MODE>
float run(std::vector<uint4*>& bufs, long bytes, int grid, int waves, hipStream_t s, unsigned* out) {
  const int copies = (int)bufs.size();
  const long pieces = bytes / 1024;
  const size_t lds = MODE == 2 ? (size_t)waves * U * 1024 : 0;
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  const int n = copies < 48 ? 48 : copies;
  for (int i = 0; i < n; ++i)
    hipLaunchKernelGGL((k_stream<U, MODE>), dim3(grid), dim3(64 * waves), lds, s, bufs[i % copies], pieces, out);
  CHECK(hipStreamEndCapture(s, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CHECK(hipGraphLaunch(ge, s));
  CHECK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0, s));
  for (int r = 0; r < 3; ++r) CHECK(hipGraphLaunch(ge, s));
  CHECK(hipEventRecord(e1, s));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  return ms * 1000.f / (3 * n);
}

int main() {
  unsigned* out;
  CHECK(hipMalloc(&out, 64));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  const char* modes[] = {"vgpr", "vgpr_nt", "lds_nt"};
  for (long mb : {8L, 23L, 46L, 117L, 235L}) {
    const long bytes = mb << 20;
    const int copies = (int)std::max(2L, std::min(48L, (6L << 30) / bytes));
    std::vector<uint4*> bufs(copies);
    for (auto& b : bufs) { CHECK(hipMalloc(&b, bytes)); CHECK(hipMemset(b, 1, bytes)); }
    for (int grid : {256, 512, 1024, 2048}) {
      for (int waves : {4, 8}) {
        for (int mode = 0; mode < 3; ++mode) {
          for (int u : {4, 8, 16}) {
            float us = 0;
#define RUN(UU, MM) us = run<UU, MM>(bufs, bytes, grid, waves, s, out)
            if (u == 4) { if (mode == 0) RUN(4, 0); else if (mode == 1) RUN(4, 1); else RUN(4, 2); }
            if (u == 8) { if (mode == 0) RUN(8, 0); else if (mode == 1) RUN(8, 1); else RUN(8, 2); }
            if (u == 16) { if (mode == 0) RUN(16, 0); else if (mode == 1) RUN(16, 1); else RUN(16, 2); }
#undef RUN
            printf("{\"MB\": %ld, \"grid\": %d, \"waves\": %d, \"mode\": \"%s\", \"U\": %d, \"us\": %.2f, \"TBps\": %.2f}\n",
                   mb, grid, waves, modes[mode], u, us, bytes / (us * 1e-6) / 1e12);
            fflush(stdout);
          }
        }
      }
    }
    for (auto& b : bufs) CHECK(hipFree(b));
  }
  return 0;
}
