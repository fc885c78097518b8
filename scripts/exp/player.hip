// Lab: does ONE persistent launch per decode layer beat separate launches at batch 1 (1x MI355X)?
//
// The post-attention chain of a TinyLlama layer (H 2048, I 5632), 22 layers of distinct weights
// (every launch streams from HBM), batch 1:
//   Wo     r += Wo . x_attn                       (2048 x 2048)
//   gate/up act = silu(Wg . n(r)) * (Wu . n(r))  (2 x 5632 x 2048, rows interleaved g0 u0 g1 u1 ..)
//   down   r += Wd . act                          (2048 x 5632)
// n(r) = r * rsqrt(mean(r^2) + eps) (norm weight folded into the weights, as the engine does).
//
//   launches : three kernels per layer (hipGraph), each wave owns the same rows as below
//   persist  : one 256-workgroup launch per layer (one workgroup per CU, one wave per SIMD), the
//              seams are grid barriers (payload: fp32 agent-scope atomic stores = sc1 write-through;
//              one monotonic counter per seam, relaxed poll + s_sleep, one agent acquire after; the
//              counters are zeroed by ONE memset node at the head of the graph), and every wave
//              issues its NEXT phase's weight rows before it waits at a seam (run-ahead in VGPRs:
//              weights do not depend on the seam)
//   persist0 : the same launch without the run-ahead (loads issued after each seam)
//   persist_xcd_seam : persist with the XCD-hierarchical seam (grid_seam_h: 8 group counters, 8
//              arrivals on the global one, per-group release flags)
// Both forms use the same row -> wave -> lane mapping and reduction order, so r must be bitwise
// equal.  Prints one JSON line per variant: us per layer.
// Build: hipcc --offload-arch=gfx950 -O3 -o expbin/player scripts/exp/player.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../../csrc/kernels/common.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int H = 2048, I = 5632, NL = 22;
constexpr int WG = 256, WPB = 4, NWAVE = WG * WPB;  // 1024 waves
constexpr int NCH = H / 512;                          // uint4 per lane for a K = 2048 row (4)
constexpr int NCI = I / 512;                          // K = 5632 -> 11
constexpr int PAIRS_MAX = (I + NWAVE - 1) / NWAVE;    // 6
constexpr float EPS = 1e-5f;

struct Layer {
  const u16* wo;   // [H, H]
  const u16* wgu;  // [2I, H] interleaved
  const u16* wd;   // [H, I]
};

__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NC>
__device__ __forceinline__ void load_row(uint4 (&w)[NC], const u16* row, int lane) {
#pragma unroll
  for (int j = 0; j < NC; ++j) w[j] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(
                                          reinterpret_cast<const u32x4*>(row + 8 * (lane + 64 * j))));
}

template <int NC>
__device__ __forceinline__ float dot_row(const uint4 (&w)[NC], const float* xs, int lane) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    float f[8];
    unpack8(w[j], f);
    const float4 a = *reinterpret_cast<const float4*>(xs + 8 * (lane + 64 * j));
    const float4 b = *reinterpret_cast<const float4*>(xs + 8 * (lane + 64 * j) + 4);
    s += f[0] * a.x + f[1] * a.y + f[2] * a.z + f[3] * a.w + f[4] * b.x + f[5] * b.y + f[6] * b.z + f[7] * b.w;
  }
  return wave_sum(s);
}

__device__ __forceinline__ float silu_mul(float g, float u) {
  const float a = g / (1.f + __expf(-g)) * u;
  return bf2f(f2bf(a));  // the engine's act is bf16
}

// stage n floats (from bf16 or f32) into LDS; returns sum of squares (block-wide) if asked
__device__ __forceinline__ void stage_bf16(float* xs, const u16* x, int n) {
  for (int i = threadIdx.x; i < n / 8; i += blockDim.x) {
    float f[8];
    unpack8(ld16(x + 8 * i), f);
#pragma unroll
    for (int q = 0; q < 8; ++q) xs[8 * i + q] = f[q];
  }
}
__device__ __forceinline__ float stage_f32_ssq(float* xs, const float* x, int n, float* red) {
  float s = 0.f;
  for (int i = threadIdx.x; i < n / 4; i += blockDim.x) {
    const float4 v = *reinterpret_cast<const float4*>(x + 4 * i);
    *reinterpret_cast<float4*>(xs + 4 * i) = v;
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  return block_sum(s, red);
}

// -------------------------------------------------------------------------- separate launches
__global__ void __launch_bounds__(256) k_wo(Layer L, const u16* xa, float* r) {
  __shared__ __attribute__((aligned(16))) float xs[H];
  const int lane = threadIdx.x & 63, gw = blockIdx.x * WPB + (threadIdx.x >> 6);
  uint4 w[2][NCH];
  load_row<NCH>(w[0], L.wo + (long)gw * H, lane);
  load_row<NCH>(w[1], L.wo + (long)(gw + NWAVE) * H, lane);
  stage_bf16(xs, xa, H);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = gw + j * NWAVE;
    const float y = dot_row<NCH>(w[j], xs, lane);
    if (lane == 0) r[row] = r[row] + y;
  }
}

__global__ void __launch_bounds__(256) k_gu(Layer L, const float* r, float* act) {
  __shared__ __attribute__((aligned(16))) float xs[H];
  __shared__ float red[16];
  const int lane = threadIdx.x & 63, gw = blockIdx.x * WPB + (threadIdx.x >> 6);
  const float ssq = stage_f32_ssq(xs, r, H, red);
  const float sc = rsqrtf(ssq / H + EPS);
  __syncthreads();
  for (int i = threadIdx.x; i < H; i += blockDim.x) xs[i] *= sc;
  __syncthreads();
  for (int j = 0; j < PAIRS_MAX; ++j) {
    const int p = gw + j * NWAVE;
    if (p >= I) break;
    uint4 wg[NCH], wu[NCH];
    load_row<NCH>(wg, L.wgu + (long)(2 * p) * H, lane);
    load_row<NCH>(wu, L.wgu + (long)(2 * p + 1) * H, lane);
    const float g = dot_row<NCH>(wg, xs, lane), u = dot_row<NCH>(wu, xs, lane);
    if (lane == 0) act[p] = silu_mul(g, u);
  }
}

__global__ void __launch_bounds__(256) k_d(Layer L, const float* act, float* r) {
  __shared__ __attribute__((aligned(16))) float xs[I];
  const int lane = threadIdx.x & 63, gw = blockIdx.x * WPB + (threadIdx.x >> 6);
  uint4 w[2][NCI];
  load_row<NCI>(w[0], L.wd + (long)gw * I, lane);
  load_row<NCI>(w[1], L.wd + (long)(gw + NWAVE) * I, lane);
  for (int i = threadIdx.x; i < I / 4; i += blockDim.x)
    *reinterpret_cast<float4*>(xs + 4 * i) = *reinterpret_cast<const float4*>(act + 4 * i);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = gw + j * NWAVE;
    const float y = dot_row<NCI>(w[j], xs, lane);
    if (lane == 0) r[row] = r[row] + y;
  }
}

// -------------------------------------------------------------------------- persistent layer
__device__ __forceinline__ void grid_seam(unsigned* ctr, unsigned* tmo) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its sc1 payload stores drained
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)WG) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {  // bounded: give up, flag it (results are then garbage)
        __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// XCD-hierarchical seam (review item 7, round 5): the 256 workgroups arrive in 8 groups of 32 (blockIdx % 8:
// the dispatcher deals workgroups to the 8 XCDs round-robin, so a group is one XCD's workgroups).  Each
// group counts its own arrivals (ctr[1 + g]); only the group's last arriver touches the global counter
// (ctr[0], 8 arrivals instead of 256) and waits for it, then raises the group's release flag
// (ctr[9 + g]) that the other 31 poll.  Same payload rules and bounded spins as grid_seam.
constexpr int SEAM_WORDS_H = 32;
__device__ __forceinline__ void grid_seam_h(unsigned* ctr, unsigned* tmo) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int g = blockIdx.x & 7;
    const unsigned prev = __hip_atomic_fetch_add(ctr + 1 + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    if (prev == (unsigned)(WG / 8) - 1) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 8u) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) { __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
      }
      __hip_atomic_store(ctr + 9 + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      while (__hip_atomic_load(ctr + 9 + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) { __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

template <bool H>
__device__ __forceinline__ void seam(unsigned* ctr, int i, unsigned* tmo) {
  if constexpr (H) grid_seam_h(ctr + i * SEAM_WORDS_H, tmo);
  else grid_seam(ctr + i * 4, tmo);
}

template <bool RUNAHEAD, bool HSEAM = false>
__global__ void __launch_bounds__(256, 1) k_layer(Layer L, const u16* xa, float* r, float* act, unsigned* bar,
                                                   unsigned* tmo) {
  __shared__ __attribute__((aligned(16))) float xs[I];
  __shared__ float red[16];
  const int lane = threadIdx.x & 63, gw = blockIdx.x * WPB + (threadIdx.x >> 6);
  constexpr int PA = 3;  // gate/up pairs loaded ahead of seam 1
  // ---- phase A: Wo (+ run-ahead of the first gate/up pairs)
  uint4 wa[2][NCH];
  load_row<NCH>(wa[0], L.wo + (long)gw * H, lane);
  load_row<NCH>(wa[1], L.wo + (long)(gw + NWAVE) * H, lane);
  uint4 wb[PA][2][NCH];
  if constexpr (RUNAHEAD) {
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int p = gw + j * NWAVE;  // j < 3: always < I
      load_row<NCH>(wb[j][0], L.wgu + (long)(2 * p) * H, lane);
      load_row<NCH>(wb[j][1], L.wgu + (long)(2 * p + 1) * H, lane);
    }
  }
  stage_bf16(xs, xa, H);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = gw + j * NWAVE;
    const float y = dot_row<NCH>(wa[j], xs, lane);
    if (lane == 0) st_agent(r + row, r[row] + y);
  }
  seam<HSEAM>(bar, 0, tmo);
  // ---- phase B: gate/up
  if constexpr (!RUNAHEAD) {
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int p = gw + j * NWAVE;
      load_row<NCH>(wb[j][0], L.wgu + (long)(2 * p) * H, lane);
      load_row<NCH>(wb[j][1], L.wgu + (long)(2 * p + 1) * H, lane);
    }
  }
  uint4 wb2[PAIRS_MAX - PA][2][NCH];
#pragma unroll
  for (int j = 0; j < PAIRS_MAX - PA; ++j) {
    const int p = gw + (PA + j) * NWAVE;
    if (p < I) {
      load_row<NCH>(wb2[j][0], L.wgu + (long)(2 * p) * H, lane);
      load_row<NCH>(wb2[j][1], L.wgu + (long)(2 * p + 1) * H, lane);
    }
  }
  const float ssq = stage_f32_ssq(xs, r, H, red);
  const float sc = rsqrtf(ssq / H + EPS);
  __syncthreads();
  for (int i = threadIdx.x; i < H; i += blockDim.x) xs[i] *= sc;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const float g = dot_row<NCH>(wb[j][0], xs, lane), u = dot_row<NCH>(wb[j][1], xs, lane);
    if (lane == 0) st_agent(act + gw + j * NWAVE, silu_mul(g, u));
  }
  uint4 wc[2][NCI];
  if constexpr (RUNAHEAD) {
    load_row<NCI>(wc[0], L.wd + (long)gw * I, lane);
    load_row<NCI>(wc[1], L.wd + (long)(gw + NWAVE) * I, lane);
  }
#pragma unroll
  for (int j = 0; j < PAIRS_MAX - PA; ++j) {
    const int p = gw + (PA + j) * NWAVE;
    if (p < I) {
      const float g = dot_row<NCH>(wb2[j][0], xs, lane), u = dot_row<NCH>(wb2[j][1], xs, lane);
      if (lane == 0) st_agent(act + p, silu_mul(g, u));
    }
  }
  seam<HSEAM>(bar, 1, tmo);
  // ---- phase C: down
  if constexpr (!RUNAHEAD) {
    load_row<NCI>(wc[0], L.wd + (long)gw * I, lane);
    load_row<NCI>(wc[1], L.wd + (long)(gw + NWAVE) * I, lane);
  }
  for (int i = threadIdx.x; i < I / 4; i += blockDim.x)
    *reinterpret_cast<float4*>(xs + 4 * i) = *reinterpret_cast<const float4*>(act + 4 * i);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = gw + j * NWAVE;
    const float y = dot_row<NCI>(wc[j], xs, lane);
    if (lane == 0) r[row] = r[row] + y;  // read by the next launch only
  }
}

// -------------------------------------------------------------------------- host
static void fill(u16* d, size_t n, unsigned seed, float scale) {
  std::vector<u16> h(n);
  unsigned s = seed;
  for (size_t i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    const float f = ((float)(s >> 8) / 16777216.f - 0.5f) * 2.f * scale;
    unsigned u;
    memcpy(&u, &f, 4);
    h[i] = (u16)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
  }
  CHECK(hipMemcpy(d, h.data(), n * 2, hipMemcpyHostToDevice));
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  std::vector<Layer> Ls(NL);
  for (int l = 0; l < NL; ++l) {
    u16 *wo, *wgu, *wd;
    CHECK(hipMalloc(&wo, (size_t)H * H * 2));
    CHECK(hipMalloc(&wgu, (size_t)2 * I * H * 2));
    CHECK(hipMalloc(&wd, (size_t)H * I * 2));
    fill(wo, (size_t)H * H, 11 + l, 0.02f);
    fill(wgu, (size_t)2 * I * H, 101 + l, 0.02f);
    fill(wd, (size_t)H * I, 1001 + l, 0.02f);
    Ls[l] = {wo, wgu, wd};
  }
  u16* xa;
  float *r, *act, *r0;
  unsigned *bar, *tmo;
  CHECK(hipMalloc(&xa, H * 2));
  fill(xa, H, 7, 1.0f);
  CHECK(hipMalloc(&r, H * 4));
  CHECK(hipMalloc(&r0, H * 4));
  CHECK(hipMalloc(&act, I * 4));
  CHECK(hipMalloc(&bar, NL * 2 * SEAM_WORDS_H * 4));
  CHECK(hipMalloc(&tmo, 4));
  CHECK(hipMemset(tmo, 0, 4));
  {
    std::vector<float> h(H);
    for (int i = 0; i < H; ++i) h[i] = sinf(0.37f * i);
    CHECK(hipMemcpy(r0, h.data(), H * 4, hipMemcpyHostToDevice));
  }
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  auto capture = [&](int mode) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    if (mode != 0) CHECK(hipMemsetAsync(bar, 0, NL * 2 * SEAM_WORDS_H * 4, st));
    for (int l = 0; l < NL; ++l) {
      if (mode == 0) {
        hipLaunchKernelGGL(k_wo, dim3(WG), dim3(256), 0, st, Ls[l], xa, r);
        hipLaunchKernelGGL(k_gu, dim3(WG), dim3(256), 0, st, Ls[l], r, act);
        hipLaunchKernelGGL(k_d, dim3(WG), dim3(256), 0, st, Ls[l], act, r);
      } else if (mode == 1) {
        hipLaunchKernelGGL((k_layer<true, false>), dim3(WG), dim3(256), 0, st, Ls[l], xa, r, act, bar + 8 * l, tmo);
      } else if (mode == 2) {
        hipLaunchKernelGGL((k_layer<false, false>), dim3(WG), dim3(256), 0, st, Ls[l], xa, r, act, bar + 8 * l, tmo);
      } else {
        hipLaunchKernelGGL((k_layer<true, true>), dim3(WG), dim3(256), 0, st, Ls[l], xa, r, act,
                           bar + 2 * SEAM_WORDS_H * l, tmo);
      }
    }
    CHECK(hipStreamEndCapture(st, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    return ge;
  };
  const char* names[4] = {"launches", "persist", "persist0", "persist_xcd_seam"};
  std::vector<float> out[4];
  float us[4];
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int mode = 0; mode < 4; ++mode) {
    hipGraphExec_t ge = capture(mode);
    // correctness pass from r0
    CHECK(hipMemcpyAsync(r, r0, H * 4, hipMemcpyDeviceToDevice, st));
    CHECK(hipGraphLaunch(ge, st));
    CHECK(hipStreamSynchronize(st));
    out[mode].resize(H);
    CHECK(hipMemcpy(out[mode].data(), r, H * 4, hipMemcpyDeviceToHost));
    // timing (r drifts; values are irrelevant to time)
    for (int w = 0; w < 3; ++w) CHECK(hipGraphLaunch(ge, st));
    CHECK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) {
      CHECK(hipMemcpyAsync(r, r0, H * 4, hipMemcpyDeviceToDevice, st));
      CHECK(hipGraphLaunch(ge, st));
    }
    CHECK(hipEventRecord(e1, st));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    us[mode] = ms * 1000.f / reps / NL;
    CHECK(hipGraphExecDestroy(ge));
  }
  unsigned htmo;
  CHECK(hipMemcpy(&htmo, tmo, 4, hipMemcpyDeviceToHost));
  for (int mode = 0; mode < 4; ++mode) {
    double md = 0, mx = 0;
    for (int i = 0; i < H; ++i) {
      md = fmax(md, fabs(out[mode][i] - out[0][i]));
      mx = fmax(mx, fabs(out[0][i]));
    }
    const bool bit = memcmp(out[mode].data(), out[0].data(), H * 4) == 0;
    printf("{\"variant\": \"%s\", \"us_per_layer\": %.2f, \"bitwise_eq_launches\": %s, \"max_abs_diff\": %.3g, "
           "\"max_abs\": %.3g, \"finite\": %s, \"timeout\": %u}\n",
           names[mode], us[mode], bit ? "true" : "false", md, mx, isfinite(mx) ? "true" : "false", htmo);
  }
  return 0;
}
