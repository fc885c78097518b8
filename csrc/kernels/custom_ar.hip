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

// The same protocol, decomposed by COLUMN SLICE so the epilogue of a row-parallel projection can
// run in it: block b owns columns [b cw, (b + 1) cw) of every row (cw = 8 tpr, tpr threads per
// row), and after the peer sum it
//   r[m, c] = bf16(bf16(sum_p y_p[m, c]) + r[m, c])   (add == 0: r = bf16(sum))
// in place and writes the row's partial sum of squares of the new r over its slice to
// ssq[b * ssq_ld + m].  This is the residual-add + RMSNorm-statistics epilogue of the TP=1 fused
// layer (tgemm EPI_RESADD) moved behind the all-reduce: the next fused GEMM (QKV / SwiGLU) folds
// the RMSNorm from these nb partial sums, so a tensor-parallel layer needs no standalone norm.
// Every rank computes the same sums in the same order: the replicated residual stays bitwise equal.
struct CarResArgs {
  const uint4* in;
  uint4* r;
  float* ssq;
  uint4* data[MAX_RANKS];
  unsigned* sig[MAX_RANKS];
  unsigned* counters;
  int* err;
  long ldr8, ssq_ld, cap8;
  int T, H8, tpr, add, rank, world;
  long spin_limit;
};

__device__ __forceinline__ unsigned car_epoch(const unsigned* counters) {
  __shared__ unsigned s_epoch;
  if (threadIdx.x == 0) s_epoch = counters[0] + 1u;
  __syncthreads();
  return s_epoch;
}

__device__ __forceinline__ void car_signal_wait(unsigned* const* sig, int rank, int world, unsigned epoch, int* err,
                                                long spin_limit) {
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid < world)
    __hip_atomic_store(sig[tid] + b * MAX_RANKS + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid < world) {
    const unsigned* s = sig[rank] + b * MAX_RANKS + tid;
    long it = 0;
    while ((int)(__hip_atomic_load(s, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(8);
      if (++it > spin_limit) {
        atomicOr(err, 1 << tid);
        break;
      }
    }
  }
  __syncthreads();
  __threadfence_system();
}

__device__ __forceinline__ void car_finish(unsigned* counters, unsigned epoch) {
  if (threadIdx.x == 0) {
    __threadfence();
    if (atomicAdd(&counters[1], 1u) == gridDim.x - 1u) {  // last block: publish the epoch
      counters[1] = 0u;
      counters[0] = epoch;
    }
  }
}

__global__ void __launch_bounds__(THREADS) car_resadd_kernel(CarResArgs a) {
  const unsigned epoch = car_epoch(a.counters);
  const long half = (long)(epoch & 1u) * a.cap8;
  const int b = blockIdx.x, tid = threadIdx.x, tpr = a.tpr, rpp = THREADS / tpr;
  const int c8 = b * tpr + tid % tpr;  // this thread's 16-B column chunk
  uint4* mine = a.data[a.rank] + half;
  for (int m = tid / tpr; m < a.T; m += rpp) mine[(long)m * a.H8 + c8] = a.in[(long)m * a.H8 + c8];
  __threadfence_system();
  __syncthreads();
  car_signal_wait(a.sig, a.rank, a.world, epoch, a.err, a.spin_limit);
  for (int m0 = 0; m0 < a.T; m0 += rpp) {
    const int m = m0 + tid / tpr;
    float ss = 0.f;
    if (m < a.T) {
      const long i = (long)m * a.H8 + c8;
      float acc[8], f[8];
      unpack8(a.data[0][half + i], acc);
      for (int p = 1; p < a.world; ++p) {
        unpack8(a.data[p][half + i], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += f[j];
      }
      uint4* rp = a.r + (long)m * a.ldr8 + c8;
      if (a.add) {
        unpack8(*rp, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = bf2f(f2bf(bf2f(f2bf(acc[j])) + f[j]));
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = bf2f(f2bf(acc[j]));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += acc[j] * acc[j];
      *rp = pack8(acc);
    }
    // row reduction over the tpr consecutive lanes of the row (tpr divides 64)
    for (int o = 1; o < tpr; o <<= 1) ss += __shfl_xor(ss, o, 64);
    if (m < a.T && tid % tpr == 0) a.ssq[(long)b * a.ssq_ld + m] = ss;
  }
  car_finish(a.counters, epoch);
}

// One-shot all-gather: out[p * n8 + i] = in_p[i] for every rank p (the vocab-parallel sampler's
// per-shard candidates), same flag protocol; block b moves the b-th strided share.
struct CarGatherArgs {
  const uint4* in;
  uint4* out;
  uint4* data[MAX_RANKS];
  unsigned* sig[MAX_RANKS];
  unsigned* counters;
  int* err;
  long n8, cap8;
  int rank, world;
  long spin_limit;
};

__global__ void __launch_bounds__(THREADS) car_gather_kernel(CarGatherArgs a) {
  const unsigned epoch = car_epoch(a.counters);
  const long half = (long)(epoch & 1u) * a.cap8;
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  uint4* mine = a.data[a.rank] + half;
  for (long i = (long)b * THREADS + tid; i < a.n8; i += (long)nb * THREADS) mine[i] = a.in[i];
  __threadfence_system();
  __syncthreads();
  car_signal_wait(a.sig, a.rank, a.world, epoch, a.err, a.spin_limit);
  for (int p = 0; p < a.world; ++p)
    for (long i = (long)b * THREADS + tid; i < a.n8; i += (long)nb * THREADS) a.out[(long)p * a.n8 + i] = a.data[p][half + i];
  car_finish(a.counters, epoch);
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

// Column-slice decomposition of [T, H]: tpr threads per row (power of two <= 64), cw = 8 tpr
// columns per block; returns the block (= ssq slot) count, < 0 if H has no valid split.
extern "C" int dllm_car_resadd_slots(int H) {
  if (H % 8) return -1;
  for (int tpr = 1; tpr <= 64; tpr <<= 1)
    if (H % (8 * tpr) == 0 && H / (8 * tpr) <= 32) return H / (8 * tpr);
  return -1;
}

extern "C" int dllm_car_resadd(const void* in, void* r, long ldr, float* ssq, long ssq_ld, int T, int H, int add,
                               void* const* bases, int world, int rank, long data_bytes, unsigned* counters, int* err,
                               long spin_limit, hipStream_t stream) {
  if (world < 1 || world > MAX_RANKS || rank < 0 || rank >= world) return -1;
  const int nb = dllm_car_resadd_slots(H);
  if (nb < 1 || ldr % 8 || (long)T * H * 2 > data_bytes || data_bytes % 16 != 0) return -2;
  if (T == 0) return nb;
  CarResArgs a{};
  a.in = (const uint4*)in;
  a.r = (uint4*)r;
  a.ssq = ssq;
  for (int p = 0; p < world; ++p) {
    a.sig[p] = (unsigned*)bases[p];
    a.data[p] = (uint4*)((char*)bases[p] + SIG_BYTES);
  }
  a.counters = counters;
  a.err = err;
  a.ldr8 = ldr / 8;
  a.ssq_ld = ssq_ld;
  a.cap8 = data_bytes / 16;
  a.T = T;
  a.H8 = H / 8;
  a.tpr = H / (8 * nb);
  a.add = add;
  a.rank = rank;
  a.world = world;
  a.spin_limit = spin_limit;
  hipLaunchKernelGGL(car_resadd_kernel, dim3(nb), dim3(THREADS), 0, stream, a);
  const int e = (int)hipGetLastError();
  return e ? -100 - e : nb;
}

extern "C" int dllm_car_allgather(const void* in, void* out, long n_bytes, void* const* bases, int world, int rank,
                                  long data_bytes, unsigned* counters, int* err, long spin_limit, hipStream_t stream) {
  if (world < 1 || world > MAX_RANKS || rank < 0 || rank >= world) return -1;
  if (n_bytes % 16 != 0 || n_bytes > data_bytes || data_bytes % 16 != 0) return -2;
  if (n_bytes == 0) return 0;
  CarGatherArgs a{};
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
  long blocks = (a.n8 + 4L * THREADS - 1) / (4L * THREADS);
  if (blocks > 32) blocks = 32;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(car_gather_kernel, dim3((int)blocks), dim3(THREADS), 0, stream, a);
  return (int)hipGetLastError();
}

// In-graph health vote glue (parallel/comm.py graph_error_flag), one launch on each side of the
// 16-byte one-shot all-reduce instead of a chain of small element-wise launches.  err[0] is the
// communicator's sticky timeout flag, err[1] the snapshot taken when the vote is staged:
//   mode 0: v[0..7] = {bf16(err[0] != 0), 0, ..., 0} (this rank's vote); err[1] = (err[0] != 0)
//   mode 1: out[0]  = err[1] ? 1                     (this rank's step data is suspect: it voted 1,
//                                                     so every rank completing the vote trips too)
//                   : err[0] ? 0                     (only the vote itself timed out: the step's own
//                                                     all-reduces were clean, and the sticky flag is
//                                                     this rank's 1 in the NEXT vote, so all ranks
//                                                     trip together one step later)
//                   : (sum v[0] > 0)                 (a peer voted 1)
// A rank never trips alone on a vote it could not complete (its sum holds stale peer halves).
namespace {
__global__ void car_vote_kernel(int mode, int* err, u16* v, int* out) {
  const int t = threadIdx.x;
  if (mode == 0) {
    const bool e = *(volatile int*)err != 0;
    if (t < 8) v[t] = (t == 0 && e) ? (u16)0x3f80 : (u16)0;
    if (t == 0) err[1] = e ? 1 : 0;
  } else if (t == 0) {
    out[0] = err[1] != 0 ? 1 : (err[0] != 0 ? 0 : (bf2f(v[0]) > 0.f ? 1 : 0));
  }
}
}  // namespace

extern "C" int dllm_car_vote(int mode, int* err, void* v, int* out, hipStream_t stream) {
  if (mode != 0 && mode != 1) return -1;
  hipLaunchKernelGGL(car_vote_kernel, dim3(1), dim3(64), 0, stream, mode, err, (u16*)v, out);
  return (int)hipGetLastError();
}
