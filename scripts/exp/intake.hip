// Per-CU intake ceiling: how many bytes per second ONE CU can pull from an L2-resident /
// MALL-resident / HBM buffer, by (a) global_load_lds (LDS-DMA, 1 KB per wave instruction) with W
// waves and D instructions in flight per wave, (b) global_load_dwordx4 into VGPRs, (c) both at
// once (half the waves each).  One workgroup per CU (grid 256), every CU streaming.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/exp/bin/intake scripts/exp/intake.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// mode 0: glds only; 1: vgpr loads only; 2: waves < W/2 glds, others vgpr
template <int W, int D, int MODE>
__global__ void __launch_bounds__(64 * W) stream_kernel(const char* __restrict__ buf, long wrap_mask, int iters,
                                                         unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[W * D * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool use_glds = MODE == 0 || (MODE == 2 && wave < W / 2);
  // each wave walks its own 1 KB pieces: piece p of (block, wave) at ((block * W + wave) * iters + p) * 1 KB
  const long base = ((long)(blockIdx.x * W + wave) * iters) * 1024;
  unsigned acc = 0;
  if (use_glds) {
    for (int p = 0; p < iters; p += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const long off = (base + (long)(p + d) * 1024 + lane * 16) & wrap_mask;
        __builtin_amdgcn_global_load_lds((const void*)(buf + off), (lds_void*)(ring + (wave * D + d) * 1024), 16, 0, 0);
      }
      vm<0>();
    }
    acc = ring[(wave * D) * 1024 + lane];
  } else {
    uint4 v[D];
    for (int p = 0; p < iters; p += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const long off = (base + (long)(p + d) * 1024 + lane * 16) & wrap_mask;
        v[d] = *reinterpret_cast<const uint4*>(buf + off);
      }
#pragma unroll
      for (int d = 0; d < D; ++d) acc ^= v[d].x ^ v[d].y ^ v[d].z ^ v[d].w;
    }
  }
  if (acc == 0x9e3779b9u) out[0] = acc;
}

// GEMM-operand pattern: each glds piece = 8 rows x 128 B at row stride `stride` bytes (lane l ->
// row l / 8, 16-B chunk l % 8); a wave walks k-steps of 128 B along its 8 rows, WGs own disjoint
// row blocks of an L2/MALL-resident matrix.
template <int W, int D, int RPI>
__global__ void __launch_bounds__(64 * W) rows_kernel(const char* __restrict__ buf, long stride, long rows_total,
                                                       int ksteps, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[W * D * 1024];
  constexpr int LPR = 64 / RPI, SEG = LPR * 16;  // lanes per row, bytes per row segment
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long row0 = ((long)(blockIdx.x * W + wave) * RPI) % rows_total;
  const char* base = buf + (row0 + lane / LPR) * stride + (lane % LPR) * 16;
  for (int p = 0; p < ksteps; p += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const long k = (long)((p + d) % (stride / SEG)) * SEG;
      __builtin_amdgcn_global_load_lds((const void*)(base + k), (lds_void*)(ring + (wave * D + d) * 1024), 16, 0, 0);
    }
    vm<0>();
  }
  if (ring[(wave * D) * 1024 + lane] == 0x5a && lane == 99) out[0] = 1;
}

template <int W, int D, int RPI>
void run_rows(const char* buf, long bytes, long stride, unsigned* out) {
  const int ksteps = 4096;
  const long rows_total = bytes / stride / 8 * 8;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((rows_kernel<W, D, RPI>), dim3(256), dim3(64 * W), 0, 0, buf, stride, rows_total, ksteps, out);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 3; ++r)
    hipLaunchKernelGGL((rows_kernel<W, D, RPI>), dim3(256), dim3(64 * W), 0, 0, buf, stride, rows_total, ksteps, out);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double total = 3.0 * 256 * W * (double)ksteps * 1024;
  printf("{\"mode\": \"rows\", \"rows_per_instr\": %d, \"bytes\": %ld, \"stride\": %ld, \"waves\": %d, \"inflight_per_wave\": %d, \"GBps_per_CU\": %.1f}\n",
         RPI, bytes, stride, W, D, total / (ms / 1000.0) / 256 / 1e9);
  fflush(stdout);
}

template <int W, int D, int MODE>
void run(const char* buf, long bytes, unsigned* out, const char* where) {
  const int iters = 4096;  // 4 MB per wave
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL((stream_kernel<W, D, MODE>), dim3(256), dim3(64 * W), 0, 0, buf, bytes - 1, iters, out);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 3; ++r)
    hipLaunchKernelGGL((stream_kernel<W, D, MODE>), dim3(256), dim3(64 * W), 0, 0, buf, bytes - 1, iters, out);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double total = 3.0 * 256 * W * (double)iters * 1024;
  const double s = ms / 1000.0;
  printf("{\"where\": \"%s\", \"mode\": \"%s\", \"waves\": %d, \"inflight_per_wave\": %d, \"GBps_per_CU\": %.1f, \"TBps_chip\": %.2f}\n",
         where, MODE == 0 ? "glds" : MODE == 1 ? "vgpr" : "mixed", W, D, total / s / 256 / 1e9, total / s / 1e12);
  fflush(stdout);
}

int main(int argc, char** argv) {
  unsigned* out;
  CHECK(hipMalloc(&out, 64));
  if (argc > 1 && std::string(argv[1]) == "rows") {
    for (long bytes : {2L << 20, 64L << 20}) {
      char* buf;
      CHECK(hipMalloc(&buf, bytes + (1 << 20)));
      CHECK(hipMemset(buf, 1, bytes + (1 << 20)));
      for (long stride : {4096L, 4352L, 4224L, 11264L, 11520L}) {
        run_rows<4, 8, 8>(buf, bytes, stride, out);
        run_rows<4, 8, 4>(buf, bytes, stride, out);
        run_rows<4, 8, 2>(buf, bytes, stride, out);
        run_rows<4, 8, 1>(buf, bytes, stride, out);
        run_rows<8, 8, 8>(buf, bytes, stride, out);
        run_rows<8, 8, 4>(buf, bytes, stride, out);
        run_rows<8, 8, 2>(buf, bytes, stride, out);
        run_rows<8, 8, 1>(buf, bytes, stride, out);
      }
      CHECK(hipFree(buf));
    }
    return 0;
  }
  struct { long bytes; const char* where; } bufs[] = {{2L << 20, "L2 (2 MB)"}, {64L << 20, "MALL (64 MB)"}, {2L << 30, "HBM (2 GB)"}};
  for (auto& b : bufs) {
    char* buf;
    CHECK(hipMalloc(&buf, b.bytes));
    CHECK(hipMemset(buf, 1, b.bytes));
    run<4, 4, 0>(buf, b.bytes, out, b.where);
    run<4, 8, 0>(buf, b.bytes, out, b.where);
    run<8, 4, 0>(buf, b.bytes, out, b.where);
    run<8, 8, 0>(buf, b.bytes, out, b.where);
    run<16, 4, 0>(buf, b.bytes, out, b.where);
    run<4, 4, 1>(buf, b.bytes, out, b.where);
    run<4, 8, 1>(buf, b.bytes, out, b.where);
    run<8, 8, 1>(buf, b.bytes, out, b.where);
    run<16, 4, 1>(buf, b.bytes, out, b.where);
    run<8, 8, 2>(buf, b.bytes, out, b.where);
    run<16, 4, 2>(buf, b.bytes, out, b.where);
    CHECK(hipFree(buf));
  }
  return 0;
}
