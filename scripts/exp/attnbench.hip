// Decode attention kernels head to head on synthetic paged KV (random block placement):
//   paged : attention.hip (16-row tile workgroups, 8 waves, LDS merge), static split grid
//   wave  : decode_attn.hip (wave-per-unit), ns = 1, 2, 4 key splits
// Prints TB/s of K/V bytes and the max |difference| between the two outputs.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/exp/bin/attnbench scripts/exp/attnbench.hip \
//          csrc/kernels/attention.hip csrc/kernels/decode_attn.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <cmath>
#include <random>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

extern "C" int dllm_paged_attention(const void* q, const void* kc, const void* vc, const int* block_tables,
                                    const int* seq_qstart, const int* seq_qlen, const int* seq_ctx,
                                    const int* tile_seq, const int* tile_tok0, void* out, float* part_o,
                                    float* part_ml, int* counters, const int* split_len, const int* items,
                                    int grid_items, int xcd_remap, int num_tiles, int nq, int nkv, int d,
                                    int max_blocks, int splits, int causal, float scale, const void* v_new, hipStream_t stream);
extern "C" int dllm_decode_attention(const void* q, const void* kc, const void* vc, const int* block_tables,
                                     const int* seq_qstart, const int* seq_ctx, const int* tile_seq, void* out,
                                     float* part_o, float* part_ml, int* counters, const int* split_len,
                                     const int* items, int grid_wgs, int num_tiles, int nq, int nkv, int d,
                                     int max_blocks, int ns, float scale, hipStream_t stream);

static uint16_t f2bf_h(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
static float bf2f_h(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
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
  const int B = argc > 1 ? atoi(argv[1]) : 512, C = argc > 2 ? atoi(argv[2]) : 2048;
  const int var = argc > 3 ? atoi(argv[3]) : 0;
  const int nq = argc > 4 ? atoi(argv[4]) : 32, nkv = argc > 5 ? atoi(argv[5]) : 4, d = argc > 6 ? atoi(argv[6]) : 64;
  std::mt19937 rng(1);
  std::vector<int> ctx(B);
  for (int i = 0; i < B; ++i)
    ctx[i] = var ? (int)(C / 4 + rng() % (unsigned)(3 * C / 2 + 1)) : C;
  std::vector<int> order(B);
  for (int i = 0; i < B; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return ctx[x] > ctx[y]; });
  const int Cm = *std::max_element(ctx.begin(), ctx.end());
  const int maxb = (Cm + 15) / 16;
  const long NB = (long)B * maxb + 8;
  const long kvel = NB * nkv * 16 * d;
  std::vector<int> perm(NB - 8);
  for (long i = 0; i < NB - 8; ++i) perm[i] = (int)i;
  std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<uint16_t> hq((long)B * nq * d), hk(kvel), hv(kvel);
  uint32_t st = 12345u;  // xorshift: uniform values in [-1, 1) (fast for GB-sized caches)
  auto uni = [&] { st ^= st << 13; st ^= st >> 17; st ^= st << 5; return (float)(st >> 8) * (2.0f / 16777216.0f) - 1.f; };
  for (auto& x : hq) x = f2bf_h(2.f * uni());
  for (long i = 0; i < kvel; ++i) { hk[i] = f2bf_h(uni()); hv[i] = f2bf_h(uni()); }
  std::vector<int> qs(B), ql(B, 1), tt(B, 0);
  for (int i = 0; i < B; ++i) qs[i] = i;
  void *q, *kc, *vc, *o1, *o2;
  int *bt, *dqs, *dql, *dcx, *dts, *dtt, *cnt;
  float *po, *pml;
  CHECK(hipMalloc(&q, hq.size() * 2)); CHECK(hipMalloc(&kc, kvel * 2)); CHECK(hipMalloc(&vc, kvel * 2));
  CHECK(hipMalloc(&o1, hq.size() * 2)); CHECK(hipMalloc(&o2, hq.size() * 2));
  CHECK(hipMalloc(&bt, (long)B * maxb * 4));
  CHECK(hipMalloc(&dqs, B * 4)); CHECK(hipMalloc(&dql, B * 4)); CHECK(hipMalloc(&dcx, B * 4));
  CHECK(hipMalloc(&dts, B * 4)); CHECK(hipMalloc(&dtt, B * 4));
  const int NSMAX = 16;
  CHECK(hipMalloc(&po, (long)B * nkv * NSMAX * 16 * d * 4)); CHECK(hipMalloc(&pml, (long)B * nkv * NSMAX * 16 * 2 * 4));
  CHECK(hipMalloc(&cnt, ((long)B * nkv + 2) * 4)); CHECK(hipMemset(cnt, 0, ((long)B * nkv + 2) * 4));
  CHECK(hipMemcpy(q, hq.data(), hq.size() * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(kc, hk.data(), kvel * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(vc, hv.data(), kvel * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(bt, perm.data(), (long)B * maxb * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dqs, qs.data(), B * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dql, ql.data(), B * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dcx, ctx.data(), B * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dts, order.data(), B * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dtt, tt.data(), B * 4, hipMemcpyHostToDevice));
  double tot = 0;
  for (int c : ctx) tot += c;
  const double bytes = tot * nkv * d * 2 * 2;
  const float scale = 1.f / sqrtf((float)d);
  auto rep = [&](const char* name, int ns, float ms) {
    printf("{\"exp\": \"attnbench\", \"kernel\": \"%s\", \"B\": %d, \"C\": %d, \"var\": %d, \"nq\": %d, \"nkv\": %d, "
           "\"d\": %d, \"ns\": %d, \"us\": %.1f, \"TBps\": %.3f}\n",
           name, B, (int)(tot / B), var, nq, nkv, d, ns, ms * 1000, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
  };
  for (int sp : {1, 2, 4}) {
    float ms = timeit([&] {
      int r = dllm_paged_attention(q, kc, vc, bt, dqs, dql, dcx, dts, dtt, o1, po, pml, cnt, nullptr, nullptr, 0, 0, B,
                                   nq, nkv, d, maxb, sp, 1, scale, nullptr, 0);
      if (r) { printf("paged rc %d\n", r); exit(1); }
    });
    rep("paged", sp, ms);
  }
  std::vector<uint16_t> r1(hq.size()), r2(hq.size());
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(r1.data(), o1, hq.size() * 2, hipMemcpyDeviceToHost));
  for (int ns : {1, 2, 4, 8}) {
    float ms = timeit([&] {
      int r = dllm_decode_attention(q, kc, vc, bt, dqs, dcx, dts, o2, po, pml, cnt, nullptr, nullptr, 0, B, nq, nkv, d,
                                    maxb, ns, scale, 0);
      if (r) { printf("wave rc %d\n", r); exit(1); }
    });
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(r2.data(), o2, hq.size() * 2, hipMemcpyDeviceToHost));
    float md = 0.f;
    for (size_t i = 0; i < r1.size(); ++i) md = std::max(md, std::fabs(bf2f_h(r1[i]) - bf2f_h(r2[i])));
    rep("wave", ns, ms);
    printf("{\"exp\": \"attnbench\", \"check\": \"wave_vs_paged\", \"ns\": %d, \"max_abs_diff\": %.5f}\n", ns, md);
  }
  // persistent work-list mode (engine path): units of ~equal key counts, longest first
  int* ditems;
  CHECK(hipMalloc(&ditems, (1 + 2L * B * nkv * NSMAX) * 4));
  const int cfgs[][2] = {{512, 256}, {2048, 256}, {4096, 256}, {4096, 128}};
  for (auto& cf : cfgs) {
    const int target = cf[0], min_chunk = cf[1];
    long chunk = std::max<long>(min_chunk, (long)((tot * nkv + target - 1) / target));
    chunk = (chunk + 31) & ~31L;
    std::vector<int> it(1, 0);
    for (int t = 0; t < B; ++t) {
      const int c = ctx[order[t]];
      const int nst = std::min<long>(NSMAX, std::max<long>(1, (c + chunk - 1) / chunk));
      for (int h = 0; h < nkv; ++h)
        for (int sp = 0; sp < nst; ++sp) { it.push_back(t | (h << 16)); it.push_back(sp | (nst << 8)); }
    }
    it[0] = (int)((it.size() - 1) / 2);
    CHECK(hipMemcpy(ditems, it.data(), it.size() * 4, hipMemcpyHostToDevice));
    {  // the engine's current path: attention.hip walking the same list with 512 workgroups
      float ms = timeit([&] {
        int r = dllm_paged_attention(q, kc, vc, bt, dqs, dql, dcx, dts, dtt, o1, po, pml, cnt, nullptr, ditems, 512, 0,
                                     B, nq, nkv, d, maxb, NSMAX, 1, scale, nullptr, 0);
        if (r) { printf("paged wl rc %d\n", r); exit(1); }
      });
      printf("{\"exp\": \"attnbench\", \"kernel\": \"paged_wl\", \"B\": %d, \"C\": %d, \"var\": %d, \"d\": %d, "
             "\"target\": %d, \"min_chunk\": %d, \"items\": %d, \"grid_wgs\": 512, \"us\": %.1f, \"TBps\": %.3f}\n",
             B, (int)(tot / B), var, d, target, min_chunk, it[0], ms * 1000, bytes / (ms * 1e-3) / 1e12);
    }
    for (int grid : {512, 1024}) {
      float ms = timeit([&] {
        int r = dllm_decode_attention(q, kc, vc, bt, dqs, dcx, dts, o2, po, pml, cnt, nullptr, ditems, grid, B, nq, nkv,
                                      d, maxb, NSMAX, scale, 0);
        if (r) { printf("wl rc %d\n", r); exit(1); }
      });
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(r2.data(), o2, hq.size() * 2, hipMemcpyDeviceToHost));
      float md = 0.f;
      for (size_t i = 0; i < r1.size(); ++i) md = std::max(md, std::fabs(bf2f_h(r1[i]) - bf2f_h(r2[i])));
      printf("{\"exp\": \"attnbench\", \"kernel\": \"wave_wl\", \"B\": %d, \"C\": %d, \"var\": %d, \"d\": %d, "
             "\"target\": %d, \"min_chunk\": %d, \"items\": %d, \"grid_wgs\": %d, \"us\": %.1f, \"TBps\": %.3f, "
             "\"max_abs_diff\": %.5f}\n",
             B, (int)(tot / B), var, d, target, min_chunk, it[0], grid, ms * 1000, bytes / (ms * 1e-3) / 1e12, md);
      fflush(stdout);
    }
  }
  return 0;
}
