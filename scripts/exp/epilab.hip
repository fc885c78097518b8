// Epilogue lab: what each fused epilogue of the production GEMM (csrc/kernels/tgemm.hip) costs
// over the PLAIN store of the same plan, at the flagship's decode batch (TinyLlama, M = 448 / 512),
// timed as hipGraph replays over rotated weight copies (every launch streams W from HBM, as one
// decode step does).  QKV = RMSNorm row scale + RoPE + paged K / V^T writes; RESADD = residual
// add in place + partial row sums of squares; SWIGLU = silu(g) * u.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/exp/bin/epilab scripts/exp/epilab.hip
// Run:   ./epilab [M]   -> one JSON line per (shape, plan, epilogue)
#include "../../csrc/kernels/tgemm.hip"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

struct Plan { int bm, bn, st, splits, ks, nw, nl; };

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 512;
  const int nq = 32, nkv = 4, d = 64, H = 2048, I = 5632, maxpos = 4096;
  struct Shape { const char* name; int N, K, epi; };
  const Shape shapes[] = {{"qkv", (nq + 2 * nkv) * d, H, dllm::EPI_QKV},
                          {"wo", H, H, dllm::EPI_RESADD},
                          {"gateup", 2 * I, H, dllm::EPI_SWIGLU},
                          {"down", H, I, dllm::EPI_RESADD}};
  const Plan plans[] = {{64, 64, 3, 1, 2, 4, 0}, {64, 128, 3, 1, 2, 8, 0}, {64, 64, 4, 1, 1, 4, 8},
                        {128, 64, 4, 1, 1, 4, 8}, {256, 128, 3, 1, 1, 8, 8}, {64, 128, 3, 2, 2, 8, 0}};
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  float *part, *ssq_in, *ssq_out, *cs;
  int *cnt, *pos, *slots, *noslots;
  CHECK(hipMalloc(&part, (64L << 20) * 4));
  CHECK(hipMalloc(&cnt, 1 << 20));
  CHECK(hipMemset(cnt, 0, 1 << 20));
  CHECK(hipMalloc(&ssq_in, 64L * M * 4));
  CHECK(hipMalloc(&ssq_out, 256L * M * 4));
  CHECK(hipMalloc(&cs, (long)maxpos * d * 4));
  CHECK(hipMalloc(&pos, M * 4));
  CHECK(hipMalloc(&slots, M * 4));
  CHECK(hipMalloc(&noslots, M * 4));
  CHECK(hipMemset(noslots, 0xff, M * 4));
  const long blocks = 8192;
  u16 *kc, *vc, *qo, *A, *Y, *vrows;
  CHECK(hipMalloc(&kc, blocks * nkv * 16 * d * 2));
  CHECK(hipMalloc(&vc, blocks * nkv * 16 * d * 2));
  CHECK(hipMalloc(&qo, (long)M * nq * d * 2));
  CHECK(hipMalloc(&vrows, (long)M * nkv * d * 2));
  CHECK(hipMalloc(&A, (long)M * I * 2));
  CHECK(hipMalloc(&Y, (long)M * 2 * I * 2));
  {
    srand(3);
    std::vector<float> h(64L * M);
    for (auto& x : h) x = 1.f + rand() / (float)RAND_MAX;
    CHECK(hipMemcpy(ssq_in, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    std::vector<float> c((long)maxpos * d);
    for (auto& x : c) x = rand() / (float)RAND_MAX;
    CHECK(hipMemcpy(cs, c.data(), c.size() * 4, hipMemcpyHostToDevice));
    std::vector<int> p(M), sl(M);
    for (int i = 0; i < M; ++i) { p[i] = rand() % maxpos; sl[i] = (int)(((long)i * 7919 % (blocks)) * 16 + rand() % 16); }
    CHECK(hipMemcpy(pos, p.data(), M * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(slots, sl.data(), M * 4, hipMemcpyHostToDevice));
    std::vector<u16> a((long)M * I);
    for (auto& x : a) { float f = rand() / (float)RAND_MAX - 0.5f; uint32_t u; memcpy(&u, &f, 4); x = u >> 16; }
    CHECK(hipMemcpy(A, a.data(), a.size() * 2, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(Y, a.data(), a.size() * 2, hipMemcpyHostToDevice));
  }
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
    for (const Plan& p : plans) {
      // variants: 0 plain, 1 plain + RMSNorm row scale (ssq partials), 2 fused epilogue,
      // 3 (QKV only) fused epilogue with every cache slot -1 (no K / V^T cache stores),
      // 4 (QKV only) V handed over row-major (v_rows, the decode form)
      for (int e = 0; e < 5; ++e) {
        if (e >= 3 && sh.epi != dllm::EPI_QKV) continue;
        if (e == 1 && sh.epi == dllm::EPI_RESADD) continue;
        const int epi = e >= 2 ? sh.epi : dllm::EPI_PLAIN;
        dllm::GemmArgs a{};
        a.A = A; a.lda = sh.K; a.M = M; a.N = sh.N; a.K = sh.K; a.splits = p.splits;
        a.kchunk = (sh.K / p.splits + 63) / 64 * 64;
        if (a.kchunk * (p.splits - 1) >= sh.K) continue;
        a.part = part; a.counters = cnt; a.W = ws[0];
        a.Y = Y; a.ldy = epi == dllm::EPI_SWIGLU ? sh.N / 2 : sh.N;
        a.ssq_in = (e >= 1 && (sh.epi == dllm::EPI_QKV || sh.epi == dllm::EPI_SWIGLU)) ? ssq_in : nullptr;
        a.ssq_in_n = 16; a.ssq_in_ld = M; a.norm_scale = 1.f / H; a.eps = 1e-5f;
        if (epi == dllm::EPI_RESADD) { a.ssq_out = ssq_out; a.ssq_out_ld = M; }
        a.pos = pos; a.cos_sin = cs; a.slots = e == 3 ? noslots : slots; a.q_out = qo; a.kc = kc; a.vc = vc;
        a.nq = nq; a.nkv = nkv; a.d = d;
        if (e == 4) { a.v_rows = vrows; a.v_ld = nkv * d; }
        const int rc = dllm_tgemm(&a, p.bm, p.bn, p.st, p.ks, p.nw, 1, epi, s, p.nl);
        if (rc != 0) continue;
        CHECK(hipStreamSynchronize(s));
        hipGraph_t g;
        hipGraphExec_t ge;
        CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < nlaunch; ++i) {
          a.W = ws[i % copies];
          dllm_tgemm(&a, p.bm, p.bn, p.st, p.ks, p.nw, 1, epi, s, p.nl);
        }
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
        const double us = ms * 1000.0 / (reps * nlaunch);
        printf("{\"M\": %d, \"shape\": \"%s\", \"N\": %d, \"K\": %d, \"plan\": \"%dx%d st%d S%d ks%d nw%d nl%d\", \"epi\": \"%s\", \"us\": %.2f, \"TFs\": %.0f}\n",
               M, sh.name, sh.N, sh.K, p.bm, p.bn, p.st, p.splits, p.ks, p.nw, p.nl,
               e == 0 ? "plain" : e == 1 ? "plain+rowscale" : e == 2 ? sh.name : e == 3 ? "qkv-no-cache-writes" : "qkv-v-rows", us,
               2.0 * M * sh.N * sh.K / us / 1e6);
        fflush(stdout);
      }
    }
    for (auto& w : ws) CHECK(hipFree(w));
  }
  return 0;
}
