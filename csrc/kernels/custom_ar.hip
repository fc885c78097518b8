// One-shot all-reduce over xGMI peer memory for latency-bound tensor-parallel messages.
//
// Decode-time TP all-reduces are B x H bf16 (8-16 KiB x B): a ring all-reduce pays 2 (w-1) link
// latencies, while on the fully connected MI355X xGMI mesh every rank can read every peer's
// buffer directly over its own point-to-point link.  Protocol (one kernel, no host sync, so it
// is hipGraph-capturable):
//   1. block b copies ITS slice of the input into this rank's IPC-shared buffer
//      (double-buffered by epoch parity),
//   2. block b publishes `epoch` into slot [b][rank] of every peer's signal array and waits until
//      every peer's slot [b][p] in its own signal array reached `epoch` (bounded spin: a missing
//      peer sets the error flag instead of hanging the GPU),
//   3. block b reads slice b from all w buffers, sums in f32 in rank order (bitwise identical on
//      every rank) and writes the output (may alias the input).
// The epoch lives in device memory (one per communicator, advanced by the last block of each
// call), so graph replays advance it.  Double buffering removes the trailing barrier: rank r
// writes half `h` again only in call e+2, which starts after r's call e+1 completed; any block of
// e+1 passing its barrier means every peer already STARTED e+1, i.e. completed call e (kernels
// are stream-ordered), so nobody still reads half `h` — whatever grid sizes the calls used.
// Buffers are allocated uncached (hipDeviceMallocUncached) so peer reads/writes over xGMI never
// see stale L2 lines; system-scope release/acquire orders data before flags.
// Same-slice-per-block across ranks is guaranteed because every rank launches the same grid for
// the same element count.
#include "common.h"

#include <cstring>

namespace {
constexpr int MAX_RANKS = 8;
constexpr int MAX_BLOCKS = 64;
constexpr int THREADS = 512;
constexpr long SIG_BYTES = 4096;  // MAX_BLOCKS x MAX_RANKS x u32, padded
static_assert(MAX_BLOCKS * MAX_RANKS * 4 <= SIG_BYTES, "signal slots must fit the signal buffer");

struct CarArgs {
  const uint4* in;
  uint4* out;
  uint4* data[MAX_RANKS];       // per rank: 2 halves of cap8 16-byte vectors
  unsigned* sig[MAX_RANKS];     // per rank: [MAX_BLOCKS][MAX_RANKS]
  unsigned* counters;           // this rank: [0] epoch of the last completed call, [1] blocks done
  int* err;
  long n8, cap8;
  int rank, world;
  long spin_limit;
};

__global__ void __launch_bounds__(THREADS) car_kernel(CarArgs a) {
  __shared__ unsigned s_epoch;
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  if (tid == 0) s_epoch = a.counters[0] + 1u;
  __syncthreads();
  const unsigned epoch = s_epoch;
  const long half = (long)(epoch & 1u) * a.cap8;
  uint4* mine = a.data[a.rank] + half;
  for (long i = (long)b * THREADS + tid; i < a.n8; i += (long)nb * THREADS) mine[i] = a.in[i];
  __threadfence_system();
  __syncthreads();
  if (tid < a.world)
    __hip_atomic_store(a.sig[tid] + b * MAX_RANKS + a.rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < a.world) {
    const unsigned* s = a.sig[a.rank] + b * MAX_RANKS + tid;
    long it = 0;
    while ((int)(__hip_atomic_load(s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(8);
      if (++it > a.spin_limit) {
        atomicOr(a.err, 1 << tid);
        break;
      }
    }
  }
  __syncthreads();
  __threadfence_system();
  for (long i = (long)b * THREADS + tid; i < a.n8; i += (long)nb * THREADS) {
    float acc[8], f[8];
    unpack8(a.data[0][half + i], acc);
    for (int p = 1; p < a.world; ++p) {
      unpack8(a.data[p][half + i], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
    a.out[i] = pack8(acc);
  }
  if (tid == 0) {
    __threadfence();
    if (atomicAdd(&a.counters[1], 1u) == (unsigned)nb - 1u) {  // last block: publish the epoch
      a.counters[1] = 0u;
      a.counters[0] = epoch;
    }
  }
}
}  // namespace

// Allocate this rank's shared region: [signals (4 KiB) | data half 0 | data half 1].
extern "C" int dllm_car_alloc(long data_bytes, void** base) {
  const long bytes = SIG_BYTES + 2 * data_bytes;
  hipError_t e = hipExtMallocWithFlags(base, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*base, 0, bytes);
}

extern "C" int dllm_car_get_handle(void* base, char* out64) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, base);
  if (e != hipSuccess) return (int)e;
  std::memcpy(out64, &h, sizeof(h) < 64 ? sizeof(h) : 64);
  return 0;
}

extern "C" int dllm_car_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

extern "C" int dllm_car_open_handle(const char* in, void** base) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, in, sizeof(h));
  return (int)hipIpcOpenMemHandle(base, h, hipIpcMemLazyEnablePeerAccess);
}

extern "C" int dllm_car_close_handle(void* base) { return (int)hipIpcCloseMemHandle(base); }
extern "C" int dllm_car_free(void* base) { return (int)hipFree(base); }

// bases[p]: rank p's region as mapped in THIS process.  n_bytes % 16 == 0, n_bytes <= data_bytes.
extern "C" int dllm_car_allreduce(const void* in, void* out, long n_bytes, void* const* bases, int world, int rank,
                                  long data_bytes, unsigned* counters, int* err, long spin_limit, hipStream_t stream) {
  if (world < 1 || world > MAX_RANKS || rank < 0 || rank >= world) return -1;
  if (n_bytes % 16 != 0 || n_bytes > data_bytes || data_bytes % 16 != 0) return -2;
  if (n_bytes == 0) return 0;
  CarArgs a{};
  a.in = (const uint4*)in;
  a.out = (uint4*)out;
  for (int p = 0; p < world; ++p) {
    a.sig[p] = (unsigned*)bases[p];
    a.data[p] = (uint4*)((char*)bases[p] + SIG_BYTES);
  }
  a.counters = counters;
  a.err = err;
  a.n8 = n_bytes / 16;
  a.cap8 = data_bytes / 16;
  a.rank = rank;
  a.world = world;
  a.spin_limit = spin_limit;
  long blocks = (a.n8 + 4L * THREADS - 1) / (4L * THREADS);  // >= 4 vectors per thread before adding blocks
  if (blocks > 32) blocks = 32;  // (<= MAX_BLOCKS signal slots)
  static_assert(32 <= MAX_BLOCKS, "grid cap within the signal slots");
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(car_kernel, dim3((int)blocks), dim3(THREADS), 0, stream, a);
  return (int)hipGetLastError();
}
