// Shared device helpers for the gfx950 (CDNA4) kernel library.
//
// Conventions used by every kernel in csrc/kernels:
//   * wave = 64 lanes; block sizes are multiples of 64;
//   * bf16 tensors are moved as 16-byte vectors (8 x bf16) — hipcc does not vectorise
//     scalar bf16 loads (cdna_hip_programming.md Guideline 13);
//   * accumulation in f32; bf16 rounding is round-to-nearest-even.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16;

struct __attribute__((aligned(16))) u16x8 { u16 v[8]; };
struct __attribute__((aligned(8))) u16x4 { u16 v[4]; };

static __device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float(((uint32_t)h) << 16); }

static __device__ __forceinline__ u16 f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (u16)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));  // inf/nan
  u += 0x7fffu + ((u >> 16) & 1u);
  return (u16)(u >> 16);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

static __device__ __forceinline__ uint4 ld16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
// non-temporal 16-B load (streamed-once operands: decode weights) -> bf16x8 operand
static __device__ __forceinline__ bf16x8 ldnt_bf16x8(const void* p) {
  return __builtin_bit_cast(bf16x8, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)));
}
static __device__ __forceinline__ void st16(void* p, uint4 v) { *reinterpret_cast<uint4*>(p) = v; }

// ---- in-launch hand-off helpers (cdna_hip_programming.md Guideline 16, recipe R1):
// payload stored WRITE-THROUGH (sc1, 16 B) so no release fence (which writes back the whole XCD
// L2) is needed; every storing wave drains with s_waitcnt vmcnt(0) before the workgroup barrier;
// one lane takes the ticket with a relaxed agent-scope atomic; the consumer reads the payload
// ONLY with sc1 loads (bypass its L1), so it needs no acquire fence either.
static __device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}
static __device__ __forceinline__ void st_wt16(__amdgpu_buffer_rsrc_t r, unsigned byte_off, float4 v) {
  const u32x4 u = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(u, r, byte_off, 0, 16 /* sc1 */);
}
static __device__ __forceinline__ float4 ld_wt16(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16 /* sc1 */);
  return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}
// Drain this wave's stores, barrier, one ticket per workgroup; returns true in the LAST arriver.
// `flag` must be a __shared__ int.  The counter is re-armed (0) by the last arriver.
static __device__ __forceinline__ bool ticket_last(int* counter, int expected, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = (old == expected - 1);
    if (last) __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

// unpack 8 bf16 (one uint4) to f32
static __device__ __forceinline__ void unpack8(uint4 v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

static __device__ __forceinline__ uint4 pack8(const float* f) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(f[2 * i]) | ((uint32_t)f2bf(f[2 * i + 1]) << 16);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

static __device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

static __device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024 (multiple of 64). `red` must hold >= 16 floats.
static __device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}
