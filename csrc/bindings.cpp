// Python bindings for the gfx950 kernel library (torch tensors -> raw launchers).
// Every entry point validates shapes/dtypes/devices on the host BEFORE launching, so a
// mis-shaped call raises instead of faulting the GPU, and launches on torch's current HIP
// stream (graph-capturable: no allocation, no sync inside).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include "kernels/tgemm_args.h"

extern "C" {
int dllm_norm(const void*, const void*, void*, const void*, const void*, void*, int, int, long, long, float, int,
              hipStream_t);
int dllm_rope_kv(const void*, long, const int*, const float*, const int*, void*, void*, void*, int, int, int, int, int,
                 hipStream_t);
int dllm_kv_write(const void*, const void*, long, const int*, void*, void*, int, int, int, int, hipStream_t);
int dllm_paged_attention(const void*, const void*, const void*, const int*, const int*, const int*, const int*,
                         const int*, const int*, void*, float*, float*, int*, const int*, const int*, int, int, int,
                         int, int, int, int, int, int, float, const void*, hipStream_t);
int dllm_silu_mul(const void*, void*, long, int, long, hipStream_t);
int dllm_embed(const int*, const void*, void*, long, int, long, long, float*, int*, const int*, int, hipStream_t);
int dllm_gemv(const void*, long, const void*, void*, long, int, int, int, int, int, const void*, void*, const void*,
              float, hipStream_t);
int dllm_gelu(const void*, void*, long, hipStream_t);
int dllm_mean_pool_l2(const void*, const int*, float*, int, int, int, hipStream_t);
int dllm_moe_gate(const float*, int, int, int, int*, float*, hipStream_t);
int dllm_moe_router(const void*, long, const void*, int, int, int, int, int*, float*, float*, hipStream_t);
int dllm_scatter_pairs(int*, const int*, int, hipStream_t);
int dllm_step_fetch(const int*, int*, int, int, int, int, const int*, const int*, int*, int, hipStream_t);
int dllm_step_store(const int*, int*, int, hipStream_t);
int dllm_argmax(const void*, long, int, int, int, int*, hipStream_t);
int dllm_sample_topp(const float*, const long*, int, int, const float*, const float*, const float*, int*, hipStream_t);
int dllm_cosine_scores(const float*, const float*, float*, int, int, int, hipStream_t);
int dllm_sample_rows(const void*, long, int, int, const float*, const float*, const int*, const unsigned*, int*,
                     hipStream_t);
int dllm_tp_cands_k();
int dllm_tp_cands(const void*, long, int, int, int, void*, hipStream_t);
int dllm_tp_sample(const void*, int, int, const float*, const float*, const int*, const unsigned*, int*, hipStream_t);
int dllm_sample_split(const void*, long, int, int, int, const float*, const float*, const int*, const unsigned*, void*,
                      long, int*, int*, hipStream_t);
int dllm_sample_split_maxp();
int dllm_sample_split_kmax();
int dllm_skinny_epi(const void*, long, const void*, int, void*, long, int, int, int, int, int, int, float*, int*, void*,
                    long, float*, long, const float*, int, long, float, float, const int*, const float*, const int*,
                    void*, void*, void*, int, int, int, hipStream_t);
int dllm_skinny_gemm(const void*, long, const void*, void*, long, int, int, int, int, int, int, float*, int*,
                     hipStream_t);
int dllm_moe_max_tiles(int, int);
int dllm_moe_ffn(const void*, long, long, int, const int*, const float*, int, int, const void*, const void*, int, int*,
                 int*, void*, float*, void*, hipStream_t);
int dllm_car_alloc(long, void**);
int dllm_car_get_handle(void*, char*);
int dllm_car_handle_size();
int dllm_car_open_handle(const char*, void**);
int dllm_car_close_handle(void*);
int dllm_car_free(void*);
int dllm_car_allreduce(const void*, void*, long, void* const*, int, int, long, unsigned*, int*, long, hipStream_t);
int dllm_car_resadd_slots(int);
int dllm_car_resadd(const void*, void*, long, float*, long, int, int, int, void* const*, int, int, long, unsigned*, int*,
                    long, hipStream_t);
int dllm_car_allgather(const void*, void*, long, void* const*, int, int, long, unsigned*, int*, long, hipStream_t);
int dllm_car_vote(int, int*, void*, int*, hipStream_t);
int dllm_tgemm(const void*, int, int, int, int, int, int, int, hipStream_t, int);
int dllm_moe_max_tiles_bm(int, int, int);
int dllm_moe_ffn_tg(const void*, long, long, int, const int*, const float*, int, int, const void*, const void*, int,
                    int*, int*, int*, void*, void*, void*, const int*, hipStream_t);
int dllm_encoder_attention(const void*, const int*, void*, int, int, int, int, float, hipStream_t);
int dllm_embed_ln(const int*, const void*, const void*, const void*, const void*, const void*, void*, int, int, int, int,
                  float, hipStream_t);
int dllm_res_add_ssq(const void*, long, void*, long, float*, long, int, int, int, hipStream_t);
int dllm_gemv_slots(int, int, int);
void dllm_gemv_set_grid(int, int, int);
int dllm_gemv_epi(const void*, long, const void*, void*, long, int, int, int, int, int, void*, long, float*, long,
                  const float*, int, long, float, float, const int*, const float*, const int*, void*, void*, void*, int,
                  int, int, hipStream_t);
int dllm_qkv_post(const void*, long, const float*, int, long, float, float, const int*, const float*, const int*, void*,
                  void*, void*, void*, int, int, int, int, hipStream_t);
int dllm_swiglu_post(const void*, long, const float*, int, long, float, float, void*, long, int, int, hipStream_t);
int dllm_flash_prefill(const void*, const void*, const void*, const int*, const int*, const int*, const int*, const int*,
                       const int*, void*, int, int, int, int, int, int, float, int, float*, float*, int*, hipStream_t);
int dllm_cache_scan(const unsigned long long*, const int*, int, const float*, const int*, long, int, float,
                    unsigned long long*, hipStream_t);
int dllm_cache_write(const unsigned long long*, const long long*, const int*, int, float*, int*, int, hipStream_t);
}

namespace {
hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_dev(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}
void check_bf16(const torch::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, name, " must be bf16");
}
void check_i32(const torch::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kInt32 && t.is_contiguous(), name, " must be contiguous int32");
}
void check_f32(const torch::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kFloat32 && t.is_contiguous(), name, " must be contiguous f32");
}
void ok(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " launch failed, code ", rc); }

// y = norm(x (+ residual)) * w (+ b); residual (if given) is updated in place to x + residual.
void norm(torch::Tensor x, c10::optional<torch::Tensor> residual, torch::Tensor w, c10::optional<torch::Tensor> b,
          torch::Tensor y, double eps, bool layernorm) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  TORCH_CHECK(x.dim() == 2 && y.dim() == 2 && x.stride(1) == 1 && y.stride(1) == 1, "x, y: 2-D row-major");
  const int rows = x.size(0), H = x.size(1);
  TORCH_CHECK(y.size(0) == rows && y.size(1) == H && w.numel() == H, "shape mismatch");
  const void* rp = nullptr;
  if (residual) {
    check_bf16(*residual, "residual");
    TORCH_CHECK(residual->is_contiguous() && residual->size(0) == rows && residual->size(1) == H, "residual shape");
    rp = residual->data_ptr();
  }
  const void* bp = nullptr;
  if (layernorm) {
    TORCH_CHECK(b.has_value(), "layernorm needs bias");
    check_bf16(*b, "b");
    bp = b->data_ptr();
  }
  ok(dllm_norm(x.data_ptr(), rp, residual ? residual->data_ptr() : nullptr, w.data_ptr(), bp, y.data_ptr(), rows, H,
               x.stride(0), y.stride(0), (float)eps, layernorm ? 1 : 0, stream()),
     "norm");
}

void rope_kv(torch::Tensor qkv, torch::Tensor pos, torch::Tensor cos_sin, torch::Tensor slots, torch::Tensor q_out,
             torch::Tensor kc, torch::Tensor vc, int64_t nq, int64_t nkv, int64_t d) {
  check_bf16(qkv, "qkv");
  check_i32(pos, "positions");
  check_f32(cos_sin, "cos_sin");
  check_i32(slots, "slot_mapping");
  check_bf16(q_out, "q_out");
  check_bf16(kc, "k_cache");
  check_bf16(vc, "v_cache");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1 && qkv.size(1) >= (nq + 2 * nkv) * d, "qkv shape");
  const int T = qkv.size(0);
  TORCH_CHECK(pos.numel() == T && slots.numel() == T, "positions/slots length");
  TORCH_CHECK(q_out.is_contiguous() && q_out.numel() == (int64_t)T * nq * d, "q_out shape");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == d, "cos_sin must be [max_pos, d]");
  TORCH_CHECK(kc.is_contiguous() && vc.is_contiguous() && kc.dim() == 4 && kc.size(1) == nkv && kc.size(2) == 16 &&
                  kc.size(3) == d && vc.size(2) == d && vc.size(3) == 16,
              "cache layout: K [blocks, nkv, 16, d], V [blocks, nkv, d, 16]");
  if (T == 0) return;
  ok(dllm_rope_kv(qkv.data_ptr(), qkv.stride(0), pos.data_ptr<int>(), cos_sin.data_ptr<float>(),
                  slots.data_ptr<int>(), q_out.data_ptr(), kc.data_ptr(), vc.data_ptr(), T, nq, nkv, d, 16, stream()),
     "rope_kv");
}

void kv_write(torch::Tensor k, torch::Tensor v, torch::Tensor slots, torch::Tensor kc, torch::Tensor vc) {
  check_bf16(k, "k");
  check_bf16(v, "v");
  check_i32(slots, "slots");
  TORCH_CHECK(k.dim() == 3 && k.is_contiguous() && v.is_contiguous() && v.sizes() == k.sizes(), "k/v [T, nkv, d]");
  const int T = k.size(0), nkv = k.size(1), d = k.size(2);
  TORCH_CHECK(kc.size(1) == nkv && kc.size(3) == d, "cache shape");
  if (T == 0) return;
  ok(dllm_kv_write(k.data_ptr(), v.data_ptr(), (long)nkv * d, slots.data_ptr<int>(), kc.data_ptr(), vc.data_ptr(), T,
                   nkv, d, 16, stream()),
     "kv_write");
}

void paged_attention(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, torch::Tensor block_tables,
                     torch::Tensor qstart, torch::Tensor qlen, torch::Tensor ctx, torch::Tensor tile_seq,
                     torch::Tensor tile_tok0, torch::Tensor out, c10::optional<torch::Tensor> part_o,
                     c10::optional<torch::Tensor> part_ml, c10::optional<torch::Tensor> counters, int64_t splits,
                     bool causal, double scale, c10::optional<torch::Tensor> split_len, bool xcd_remap,
                     c10::optional<torch::Tensor> items, int64_t grid_items, c10::optional<torch::Tensor> v_new) {
  check_bf16(q, "q");
  check_bf16(kc, "k_cache");
  check_bf16(vc, "v_cache");
  check_bf16(out, "out");
  for (auto* t : {&block_tables, &qstart, &qlen, &ctx, &tile_seq, &tile_tok0}) check_i32(*t, "attention metadata");
  TORCH_CHECK(q.dim() == 3 && q.is_contiguous() && out.is_contiguous() && out.sizes() == q.sizes(), "q/out [T, nq, d]");
  const int nq = q.size(1), d = q.size(2);
  TORCH_CHECK(kc.dim() == 4 && kc.size(2) == 16 && kc.size(3) == d && vc.size(2) == d && vc.size(3) == 16,
              "cache layout");
  const int nkv = kc.size(1);
  TORCH_CHECK(nq % nkv == 0 && 16 % (nq / nkv) == 0, "GQA group must divide 16");
  TORCH_CHECK(d == 64 || d == 96 || d == 128, "head_dim must be 64, 96 or 128");
  TORCH_CHECK(block_tables.dim() == 2, "block_tables [num_seqs, max_blocks]");
  const int num_seqs = block_tables.size(0);
  TORCH_CHECK(qstart.numel() == num_seqs && qlen.numel() == num_seqs && ctx.numel() == num_seqs, "seq metadata len");
  const int num_tiles = tile_seq.numel();
  TORCH_CHECK(tile_tok0.numel() == num_tiles, "tile metadata len");
  float* po = nullptr;
  float* pml = nullptr;
  int* cnt = nullptr;
  if (splits > 1) {
    TORCH_CHECK(counters.has_value(), "split-K needs a zeroed counter buffer");
    check_i32(*counters, "counters");
    TORCH_CHECK(counters->numel() >= (int64_t)num_tiles * nkv, "counter buffer too small");
    cnt = counters->data_ptr<int>();
    TORCH_CHECK(part_o.has_value() && part_ml.has_value(), "split-K needs workspaces");
    check_f32(*part_o, "part_o");
    check_f32(*part_ml, "part_ml");
    TORCH_CHECK(part_o->numel() >= (int64_t)num_tiles * nkv * splits * 16 * d &&
                    part_ml->numel() >= (int64_t)num_tiles * nkv * splits * 16 * 2,
                "workspace too small");
    po = part_o->data_ptr<float>();
    pml = part_ml->data_ptr<float>();
  }
  const int* sl = nullptr;
  if (split_len.has_value()) {
    check_i32(*split_len, "split_len");
    TORCH_CHECK(split_len->numel() >= 1, "split_len: device scalar");
    sl = split_len->data_ptr<int>();
  }
  const int* it = nullptr;
  if (items.has_value()) {
    // work list [1 + 2 * n]: units outside (num_tiles, nkv, splits) are skipped by the kernel; the
    // two ints after the tile counters hold the dynamic-fetch cursor and exit count (kept zeroed)
    check_i32(*items, "items");
    TORCH_CHECK(splits > 1 && cnt != nullptr, "work-list attention needs split-K workspaces");
    TORCH_CHECK(items->numel() >= 1, "work list [1 + 2n]");
    TORCH_CHECK(counters->numel() >= (int64_t)num_tiles * nkv + 2, "work list: counters need 2 cursor slots");
    TORCH_CHECK(grid_items >= 1 && !xcd_remap, "work-list attention: grid >= 1, no XCD remap");
    it = items->data_ptr<int>();
  }
  const void* vn = nullptr;
  if (v_new.has_value()) {   // decode: the newest token's V row-major [T, nkv * d] (tgemm v_rows)
    check_bf16(*v_new, "v_new");
    TORCH_CHECK(v_new->is_contiguous() && v_new->numel() >= (int64_t)q.size(0) * nkv * d, "v_new [T, nkv * d]");
    vn = v_new->data_ptr();
  }
  ok(dllm_paged_attention(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), block_tables.data_ptr<int>(),
                          qstart.data_ptr<int>(), qlen.data_ptr<int>(), ctx.data_ptr<int>(), tile_seq.data_ptr<int>(),
                          tile_tok0.data_ptr<int>(), out.data_ptr(), po, pml, cnt, sl, it, (int)grid_items,
                          xcd_remap ? 1 : 0, num_tiles, nq, nkv, d, block_tables.size(1), splits, causal ? 1 : 0,
                          (float)scale, vn, stream()),
     "paged_attention");
}

// Flash-style prefill attention (csrc/kernels/flash_prefill.hip): 256-row GQA tiles with K/V
// staged once per workgroup in LDS.  tile_seq/tile_tok0 hold 256 / G tokens per tile.
void flash_prefill(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, torch::Tensor block_tables,
                   torch::Tensor qstart, torch::Tensor qlen, torch::Tensor ctx, torch::Tensor tile_seq,
                   torch::Tensor tile_tok0, torch::Tensor out, bool causal, double scale, int64_t splits,
                   c10::optional<torch::Tensor> part_o, c10::optional<torch::Tensor> part_ml,
                   c10::optional<torch::Tensor> counters) {
  check_bf16(q, "q");
  check_bf16(kc, "k_cache");
  check_bf16(vc, "v_cache");
  check_bf16(out, "out");
  for (auto* t : {&block_tables, &qstart, &qlen, &ctx, &tile_seq, &tile_tok0}) check_i32(*t, "attention metadata");
  TORCH_CHECK(q.dim() == 3 && q.is_contiguous() && out.is_contiguous() && out.sizes() == q.sizes(), "q/out [T, nq, d]");
  const int nq = q.size(1), d = q.size(2);
  TORCH_CHECK(d == 64 || d == 96 || d == 128, "flash prefill: head_dim 64, 96 or 128");
  TORCH_CHECK(kc.is_contiguous() && vc.is_contiguous() && kc.dim() == 4 && kc.size(2) == 16 && kc.size(3) == d &&
                  vc.size(2) == d && vc.size(3) == 16,
              "cache layout");
  const int nkv = kc.size(1);
  TORCH_CHECK(nq % nkv == 0 && 128 % (nq / nkv) == 0, "GQA group must divide 128");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(1) >= 1, "block_tables [S, max_blocks]");
  const int S = block_tables.size(0);
  TORCH_CHECK(qstart.numel() == S && qlen.numel() == S && ctx.numel() == S, "seq metadata len");
  TORCH_CHECK(tile_tok0.numel() == tile_seq.numel(), "tile metadata len");
  float* po = nullptr;
  float* pml = nullptr;
  int* cnt = nullptr;
  if (splits > 1) {
    TORCH_CHECK(splits <= 16 && part_o.has_value() && part_ml.has_value() && counters.has_value(),
                "flash_prefill: split-KV needs part_o / part_ml / counters, splits <= 16");
    const long units = (long)tile_seq.numel() * nkv * splits;
    check_f32(*part_o, "part_o");
    check_f32(*part_ml, "part_ml");
    check_i32(*counters, "counters");
    TORCH_CHECK(part_o->numel() >= units * 256 * d && part_ml->numel() >= units * 256 * 4 &&
                    counters->numel() >= (long)tile_seq.numel() * nkv,
                "flash_prefill: split-KV workspace too small");
    po = part_o->data_ptr<float>();
    pml = part_ml->data_ptr<float>();
    cnt = counters->data_ptr<int>();
  }
  ok(dllm_flash_prefill(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), block_tables.data_ptr<int>(), qstart.data_ptr<int>(),
                        qlen.data_ptr<int>(), ctx.data_ptr<int>(), tile_seq.data_ptr<int>(), tile_tok0.data_ptr<int>(),
                        out.data_ptr(), tile_seq.numel(), nq, nkv, d, block_tables.size(1), causal ? 1 : 0,
                        (float)scale, (int)std::max<int64_t>(1, splits), po, pml, cnt, stream()),
     "flash_prefill");
}

void silu_mul(torch::Tensor gu, torch::Tensor out) {
  check_bf16(gu, "gate_up");
  check_bf16(out, "out");
  TORCH_CHECK(gu.dim() == 2 && gu.stride(1) == 1 && out.is_contiguous(), "2-D row-major");
  const long T = gu.size(0);
  const int I = gu.size(1) / 2;
  TORCH_CHECK(out.size(0) == T && out.size(1) == I, "out shape");
  ok(dllm_silu_mul(gu.data_ptr(), out.data_ptr(), T, I, gu.stride(0), stream()), "silu_mul");
}

// token-embedding gather; ssq (optional, f32 [>= T]): each row's sum of squares
// sc_dst / sc_buf (optional, int32): a decode step's block-table updates (scatter_pairs layout),
// applied by one extra workgroup of the same launch.
void embed(torch::Tensor ids, torch::Tensor table, torch::Tensor out, int64_t lo, c10::optional<torch::Tensor> ssq,
           c10::optional<torch::Tensor> sc_dst, c10::optional<torch::Tensor> sc_buf) {
  TORCH_CHECK(ids.scalar_type() == torch::kInt && ids.is_contiguous() && ids.is_cuda(), "ids: contiguous int32");
  check_bf16(table, "table");
  check_bf16(out, "out");
  TORCH_CHECK(table.dim() == 2 && table.is_contiguous() && out.is_contiguous(), "table [rows, H] contiguous");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == ids.numel() && out.size(1) == table.size(1), "out [T, H]");
  float* sp = nullptr;
  if (ssq.has_value()) {
    check_f32(*ssq, "ssq");
    TORCH_CHECK(ssq->is_contiguous() && ssq->numel() >= ids.numel(), "ssq [>= T] contiguous");
    sp = ssq->data_ptr<float>();
  }
  int* dst = nullptr;
  const int* buf = nullptr;
  int cap = 0;
  if (sc_buf.has_value()) {
    TORCH_CHECK(sc_dst.has_value(), "embed: sc_buf needs sc_dst");
    for (auto* t : {&*sc_dst, &*sc_buf})
      TORCH_CHECK(t->scalar_type() == torch::kInt && t->is_contiguous() && t->is_cuda(), "embed: scatter operands int32");
    dst = sc_dst->data_ptr<int>();
    buf = sc_buf->data_ptr<int>();
    cap = (int)((sc_buf->numel() - 1) / 2);
  }
  ok(dllm_embed(ids.data_ptr<int>(), table.data_ptr(), out.data_ptr(), ids.numel(), table.size(1), lo,
                table.size(0), sp, dst, buf, cap, stream()),
     "embed");
}

void gelu(torch::Tensor x, torch::Tensor y) {
  check_bf16(x, "x");
  check_bf16(y, "y");
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel(), "contiguous same-size");
  ok(dllm_gelu(x.data_ptr(), y.data_ptr(), x.numel(), stream()), "gelu");
}

void mean_pool_l2(torch::Tensor x, torch::Tensor lens, torch::Tensor out) {
  check_bf16(x, "x");
  check_i32(lens, "lens");
  check_f32(out, "out");
  TORCH_CHECK(x.dim() == 3 && x.is_contiguous(), "x [B, S, H]");
  const int B = x.size(0), S = x.size(1), H = x.size(2);
  TORCH_CHECK(lens.numel() == B && out.size(0) == B && out.size(1) == H, "shapes");
  ok(dllm_mean_pool_l2(x.data_ptr(), lens.data_ptr<int>(), out.data_ptr<float>(), B, S, H, stream()), "mean_pool_l2");
}

void moe_gate(torch::Tensor logits, int64_t k, torch::Tensor ids, torch::Tensor w) {
  check_f32(logits, "router_logits");
  check_i32(ids, "ids");
  check_f32(w, "weights");
  const int T = logits.size(0), E = logits.size(1);
  TORCH_CHECK(ids.numel() == (int64_t)T * k && w.numel() == (int64_t)T * k, "out shapes");
  ok(dllm_moe_gate(logits.data_ptr<float>(), T, E, k, ids.data_ptr<int>(), w.data_ptr<float>(), stream()), "moe_gate");
}

// fused router GEMV + top-k (batch-invariant): x [T, H] (row stride % 8), wg [E, H] -> ids/w [T, k]
void moe_router(torch::Tensor x, torch::Tensor wg, int64_t k, torch::Tensor ids, torch::Tensor w,
                c10::optional<torch::Tensor> logits) {
  check_bf16(x, "x");
  check_bf16(wg, "router weight");
  check_i32(ids, "ids");
  check_f32(w, "weights");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && wg.dim() == 2 && wg.is_contiguous() && wg.size(1) == x.size(1),
              "x [T, H] row-major, wg [E, H] contiguous");
  const int T = x.size(0), E = wg.size(0), H = x.size(1);
  TORCH_CHECK(ids.numel() == (int64_t)T * k && w.numel() == (int64_t)T * k && ids.is_contiguous() && w.is_contiguous(),
              "out shapes");
  float* lp = nullptr;
  if (logits.has_value()) {
    check_f32(*logits, "logits");
    TORCH_CHECK(logits->is_contiguous() && logits->numel() == (int64_t)T * E, "logits [T, E]");
    lp = logits->data_ptr<float>();
  }
  ok(dllm_moe_router(x.data_ptr(), x.stride(0), wg.data_ptr(), T, E, H, k, ids.data_ptr<int>(), w.data_ptr<float>(),
                     lp, stream()),
     "moe_router");
}

// dst (int32, any shape, contiguous) flat[idx_i] = val_i for buf = [n, idx0, val0, ...]
// Device address of a pinned (hipHostMalloc'd) host tensor, for kernels that read / write it.
static void* mapped_ptr(const torch::Tensor& t, const char* what) {
  TORCH_CHECK(t.device().is_cpu() && t.is_pinned() && t.is_contiguous() && t.scalar_type() == torch::kInt,
              what, ": pinned contiguous int32 host tensor");
  void* dptr = nullptr;
  ok((int)hipHostGetDevicePointer(&dptr, t.data_ptr(), 0), what);
  return dptr;
}

// Decode-step inputs from the pinned staging buffer (device-mapped) into dec_dev, with the
// pipelined id gather (ids[i] = d_out[src[i]] where src[i] >= 0) and the attention work list.
void step_fetch(torch::Tensor dec_host, torch::Tensor dec_dev, int64_t ids_off, int64_t src_off, int64_t n_ids,
                torch::Tensor d_out, c10::optional<torch::Tensor> items_host, c10::optional<torch::Tensor> items_dev) {
  TORCH_CHECK(dec_dev.is_cuda() && dec_dev.scalar_type() == torch::kInt && dec_dev.is_contiguous() &&
                  dec_dev.numel() == dec_host.numel(), "step_fetch: dec_dev int32 like dec_host");
  TORCH_CHECK(d_out.is_cuda() && d_out.scalar_type() == torch::kInt && d_out.numel() > n_ids, "step_fetch: d_out");
  const int* ih = nullptr;
  int* idv = nullptr;
  int cap = 0;
  if (items_host.has_value()) {
    TORCH_CHECK(items_dev.has_value() && items_dev->is_cuda() && items_dev->scalar_type() == torch::kInt &&
                    items_dev->numel() >= items_host->numel(), "step_fetch: items_dev");
    ih = (const int*)mapped_ptr(*items_host, "step_fetch items_host");
    idv = items_dev->data_ptr<int>();
    cap = (int)items_host->numel();
  }
  ok(dllm_step_fetch((const int*)mapped_ptr(dec_host, "step_fetch dec_host"), dec_dev.data_ptr<int>(),
                     (int)dec_host.numel(), (int)ids_off, (int)src_off, (int)n_ids, d_out.data_ptr<int>(), ih, idv, cap,
                     stream()),
     "step_fetch");
}

// out_host[0:n] <- d_out[0:n] by a kernel (last node of a decode-step graph).
void step_store(torch::Tensor d_out, torch::Tensor out_host, int64_t n) {
  TORCH_CHECK(d_out.is_cuda() && d_out.scalar_type() == torch::kInt && d_out.numel() >= n && out_host.numel() >= n,
              "step_store: shapes");
  ok(dllm_step_store(d_out.data_ptr<int>(), (int*)mapped_ptr(out_host, "step_store out_host"), (int)n, stream()),
     "step_store");
}

void scatter_pairs(torch::Tensor dst, torch::Tensor buf) {
  check_i32(dst, "dst");
  check_i32(buf, "buf");
  TORCH_CHECK(buf.numel() >= 1 && buf.numel() % 2 == 1, "buf = [n, (idx, val)*]");
  ok(dllm_scatter_pairs(dst.data_ptr<int>(), buf.data_ptr<int>(), (int)(buf.numel() - 1) / 2, stream()),
     "scatter_pairs");
}

void argmax(torch::Tensor logits, torch::Tensor out) {
  check_dev(logits, "logits");
  check_i32(out, "out");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits [B, V] row-major");
  const bool bf = logits.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == torch::kFloat32, "logits bf16 or f32");
  TORCH_CHECK(logits.stride(0) % (bf ? 8 : 4) == 0, "row stride must keep 16-B alignment");
  TORCH_CHECK(out.numel() == logits.size(0), "out len");
  ok(dllm_argmax(logits.data_ptr(), logits.stride(0), logits.size(0), logits.size(1), bf ? 1 : 0,
                 out.data_ptr<int>(), stream()),
     "argmax");
}

void sample_topp(torch::Tensor vals, torch::Tensor idx, torch::Tensor temp, torch::Tensor top_p, torch::Tensor u,
                 torch::Tensor out) {
  check_f32(vals, "vals");
  check_dev(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == torch::kInt64 && idx.is_contiguous(), "idx int64");
  check_f32(temp, "temperature");
  check_f32(top_p, "top_p");
  check_f32(u, "uniform");
  check_i32(out, "out");
  const int B = vals.size(0), K = vals.size(1);
  TORCH_CHECK(idx.size(0) == B && idx.size(1) == K && temp.numel() == B && top_p.numel() == B && u.numel() == B &&
                  out.numel() == B,
              "shapes");
  ok(dllm_sample_topp(vals.data_ptr<float>(), (const long*)idx.data_ptr<int64_t>(), B, K, temp.data_ptr<float>(),
                      top_p.data_ptr<float>(), u.data_ptr<float>(), out.data_ptr<int>(), stream()),
     "sample_topp");
}

// Fused per-row sampler: temp <= 0 -> arg-max; else exact top-k (k <= 256; 0 -> 256), temperature,
// top-p and an inverse-CDF draw with u = hash(seed, row).  seed: int32 device scalar.
void sample_rows(torch::Tensor logits, torch::Tensor temp, torch::Tensor top_p, torch::Tensor top_k,
                 torch::Tensor seed, torch::Tensor out) {
  check_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.stride(0) % 8 == 0,
              "logits [B, V] row-major, 16-B aligned rows");
  check_f32(temp, "temperature");
  check_f32(top_p, "top_p");
  check_i32(top_k, "top_k");
  check_i32(seed, "seed");
  check_i32(out, "out");
  const int B = logits.size(0);
  TORCH_CHECK(temp.numel() >= B && top_p.numel() >= B && top_k.numel() >= B && out.numel() >= B &&
                  seed.numel() >= 1,
              "per-row parameter lengths");
  ok(dllm_sample_rows(logits.data_ptr(), logits.stride(0), B, logits.size(1), temp.data_ptr<float>(),
                      top_p.data_ptr<float>(), top_k.data_ptr<int>(), (const unsigned*)seed.data_ptr<int>(),
                      out.data_ptr<int>(), stream()),
     "sample_rows");
}

// Split-vocab sampler for small batches: grid (P shards, B rows), same tokens as sample_rows.
// part: f32/int32 workspace >= B * P * KMAX * 2 elements; counters: int32 >= B, zero (re-armed).
int64_t sample_split_maxp() { return dllm_sample_split_maxp(); }
int64_t sample_split_kmax() { return dllm_sample_split_kmax(); }
void sample_split(torch::Tensor logits, torch::Tensor temp, torch::Tensor top_p, torch::Tensor top_k,
                  torch::Tensor seed, torch::Tensor part, torch::Tensor counters, torch::Tensor out, int64_t P) {
  check_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.stride(0) % 8 == 0,
              "logits [B, V] row-major, 16-B aligned rows");
  check_f32(temp, "temperature");
  check_f32(top_p, "top_p");
  check_i32(top_k, "top_k");
  check_i32(seed, "seed");
  check_i32(out, "out");
  check_i32(counters, "counters");
  const int B = logits.size(0);
  TORCH_CHECK(temp.numel() >= B && top_p.numel() >= B && top_k.numel() >= B && out.numel() >= B &&
                  seed.numel() >= 1 && counters.numel() >= B,
              "per-row parameter lengths");
  TORCH_CHECK(part.is_cuda() && part.is_contiguous() && part.element_size() == 4, "part: 4-byte workspace");
  TORCH_CHECK(P >= 1 && P <= dllm_sample_split_maxp(), "shards P");
  ok(dllm_sample_split(logits.data_ptr(), logits.stride(0), B, logits.size(1), (int)P, temp.data_ptr<float>(),
                       top_p.data_ptr<float>(), top_k.data_ptr<int>(), (const unsigned*)seed.data_ptr<int>(),
                       part.data_ptr(), (long)part.numel() * 4, counters.data_ptr<int>(), out.data_ptr<int>(), stream()),
     "sample_split");
}

// vocab-parallel sampler (csrc/kernels/sampling.hip): a shard's ranked top-KC candidates as int32
// pairs (value f32 bits, global id) [S, KC, 2], and the merge + draw over all-gathered [tp, S, KC, 2]
int64_t tp_cands_k() { return dllm_tp_cands_k(); }
void tp_cands(torch::Tensor logits, int64_t start, torch::Tensor cand) {
  check_bf16(logits, "logits");
  check_i32(cand, "cand");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && logits.stride(0) % 8 == 0,
              "logits [S, V] row-major, 16-B aligned rows");
  const int S = logits.size(0), KC = dllm_tp_cands_k();
  TORCH_CHECK(cand.is_contiguous() && cand.numel() == (int64_t)S * KC * 2, "cand [S, KC, 2] int32");
  ok(dllm_tp_cands(logits.data_ptr(), logits.stride(0), S, logits.size(1), (int)start, cand.data_ptr(), stream()),
     "tp_cands");
}
void tp_sample(torch::Tensor cands, torch::Tensor temp, torch::Tensor top_p, torch::Tensor top_k, torch::Tensor seed,
               torch::Tensor out) {
  check_i32(cands, "cands");
  check_f32(temp, "temperature");
  check_f32(top_p, "top_p");
  check_i32(top_k, "top_k");
  check_i32(seed, "seed");
  check_i32(out, "out");
  const int KC = dllm_tp_cands_k();
  TORCH_CHECK(cands.is_contiguous() && cands.dim() == 4 && cands.size(2) == KC && cands.size(3) == 2 &&
                  cands.size(0) >= 1 && cands.size(0) <= 8,
              "cands [tp <= 8, S, KC, 2] int32");
  const int tp = cands.size(0), S = cands.size(1);
  TORCH_CHECK(temp.numel() >= S && top_p.numel() >= S && top_k.numel() >= S && out.numel() >= S && seed.numel() >= 1,
              "per-row parameter lengths");
  ok(dllm_tp_sample(cands.data_ptr(), S, tp, temp.data_ptr<float>(), top_p.data_ptr<float>(), top_k.data_ptr<int>(),
                    (const unsigned*)seed.data_ptr<int>(), out.data_ptr<int>(), stream()),
     "tp_sample");
}

void cosine_scores(torch::Tensor q, torch::Tensor c, torch::Tensor s) {
  check_f32(q, "q");
  check_f32(c, "c");
  check_f32(s, "s");
  TORCH_CHECK(q.dim() == 2 && c.dim() == 2 && q.size(1) == c.size(1), "q [B,d], c [N,d]");
  TORCH_CHECK(s.size(0) == q.size(0) && s.size(1) == c.size(0), "s [B,N]");
  ok(dllm_cosine_scores(q.data_ptr<float>(), c.data_ptr<float>(), s.data_ptr<float>(), q.size(0), c.size(0),
                        q.size(1), stream()),
     "cosine_scores");
}

// one launch for up to 128 semantic-cache lookups (csrc/kernels/cosine.hip cache_scan_kernel):
// qptrs = device addresses of the queries' f32 [d] vectors (kept alive by the caller), qcids = their
// context ids; best[i] <- packed (orderable sim << 32 | ~row) key, 0 = no row >= thr
void cache_scan(std::vector<int64_t> qptrs, std::vector<int64_t> qcids, torch::Tensor table, torch::Tensor ctx,
                int64_t n_rows, double thr, torch::Tensor best) {
  check_f32(table, "table");
  check_i32(ctx, "ctx");
  check_dev(best, "best");
  TORCH_CHECK(table.dim() == 2 && table.size(1) % 4 == 0 && table.size(1) <= 1024, "table [N, d], d % 4 == 0, d <= 1024");
  TORCH_CHECK(n_rows >= 0 && n_rows <= table.size(0) && ctx.numel() >= n_rows, "rows within table/ctx");
  TORCH_CHECK(n_rows < 0xffffffffLL, "row index must fit the 32-bit key");
  const int nq = (int)qptrs.size();
  TORCH_CHECK(nq >= 1 && nq <= 128 && (int)qcids.size() == nq, "1..128 queries with one context id each");
  TORCH_CHECK(best.scalar_type() == torch::kInt64 && best.is_contiguous() && best.numel() >= nq, "best: int64[nq]");
  std::vector<unsigned long long> qp(nq);
  std::vector<int> qc(nq);
  for (int i = 0; i < nq; ++i) {
    TORCH_CHECK(qptrs[i] != 0 && (qptrs[i] & 15) == 0, "query vectors must be 16-B aligned device memory");
    qp[i] = (unsigned long long)qptrs[i];
    qc[i] = (int)qcids[i];
  }
  ok(dllm_cache_scan(qp.data(), qc.data(), nq, table.data_ptr<float>(), ctx.data_ptr<int>(), (long)n_rows,
                     (int)table.size(1), (float)thr, (unsigned long long*)best.data_ptr<int64_t>(), stream()),
     "cache_scan");
}

// deferred routing-cache table writes, <= 64 per launch: row slots[i] <- f32 [d] at srcs[i] (0: keep),
// ctx[slots[i]] <- cids[i]
void cache_write(std::vector<int64_t> srcs, std::vector<int64_t> slots, std::vector<int64_t> cids, torch::Tensor table,
                 torch::Tensor ctx) {
  check_f32(table, "table");
  check_i32(ctx, "ctx");
  const int n = (int)srcs.size();
  TORCH_CHECK(n <= 64 && (int)slots.size() == n && (int)cids.size() == n, "<= 64 writes");
  std::vector<unsigned long long> sp(n);
  std::vector<long long> sl(n);
  std::vector<int> ci(n);
  for (int i = 0; i < n; ++i) {
    TORCH_CHECK(slots[i] >= 0 && slots[i] < table.size(0) && slots[i] < ctx.numel(), "slot out of range");
    TORCH_CHECK((srcs[i] & 15) == 0, "source vectors must be 16-B aligned");
    sp[i] = (unsigned long long)srcs[i];
    sl[i] = slots[i];
    ci[i] = (int)cids[i];
  }
  ok(dllm_cache_write(sp.data(), sl.data(), ci.data(), n, table.data_ptr<float>(), ctx.data_ptr<int>(),
                      (int)table.size(1), stream()),
     "cache_write");
}
// y[M, N] = x[M, K] . w[N, K]^T   (swiglu: x is [M, 2K] gate|up, silu(gate)*up computed on load)
void skinny_gemm(torch::Tensor x, torch::Tensor w, torch::Tensor y, int64_t ntw, int64_t splits, bool swiglu,
                 torch::Tensor part, torch::Tensor counters) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  check_f32(part, "part");
  check_i32(counters, "counters");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && w.dim() == 2 && w.is_contiguous() && y.dim() == 2 &&
                  y.stride(1) == 1,
              "2-D row-major operands");
  const int M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(x.size(1) == (swiglu ? 2 * K : K), "x inner dim");
  TORCH_CHECK(y.size(0) == M && y.size(1) == N, "y shape");
  TORCH_CHECK(M >= 1 && M <= 128 && K % 32 == 0, "M in [1,128], K % 32 == 0");
  TORCH_CHECK(ntw == 1 || ntw == 2 || ntw == 4, "ntw in {1,2,4}");
  // slab rows = the kernel's row-tile height (MT x 16, MT in {1, 2, 4, 8}), not ceil(M / 16) x 16
  const int nc = 16 * ntw, tiles = (N + nc - 1) / nc,
            mp = 16 * (M <= 16 ? 1 : M <= 32 ? 2 : M <= 64 ? 4 : 8);
  if (splits > 1) {
    TORCH_CHECK(part.numel() >= (int64_t)splits * tiles * nc * mp, "split-K workspace too small");
    TORCH_CHECK(counters.numel() >= tiles, "counter buffer too small");
  }
  ok(dllm_skinny_gemm(x.data_ptr(), x.stride(0), w.data_ptr(), y.data_ptr(), y.stride(0), M, N, K, ntw, splits, swiglu ? 1 : 0,
        part.data_ptr<float>(), counters.data_ptr<int>(), stream()),
     "skinny_gemm");
}
// Small-batch (M <= 16) MFMA GEMM with a fused decoder epilogue (csrc/kernels/skinny_gemm.hip
// skinny_epi_kernel): epi 0 plain (y), 1 residual add (res in place + per-tile row sums -> ssq_out),
// 2 QKV (RoPE, q_out, paged K / V^T), 3 SwiGLU (y = act [M, N/2]).  w: [N, K] or the panel copy
// [K/64, N, 64].  Returns the row-sum slots written (RESADD) or 0.
int64_t skinny_epi(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> y, int64_t ntw, int64_t splits,
                   int64_t epi, torch::Tensor part, torch::Tensor counters, c10::optional<torch::Tensor> res,
                   c10::optional<torch::Tensor> ssq_out, c10::optional<torch::Tensor> ssq_in, int64_t ssq_n,
                   double scale, double eps, c10::optional<torch::Tensor> pos, c10::optional<torch::Tensor> cos_sin,
                   c10::optional<torch::Tensor> slots, c10::optional<torch::Tensor> q_out,
                   c10::optional<torch::Tensor> kc, c10::optional<torch::Tensor> vc, int64_t nq, int64_t nkv, int64_t d) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_f32(part, "part");
  check_i32(counters, "counters");
  const bool panel = w.dim() == 3;
  TORCH_CHECK(((w.dim() == 2) || (panel && w.size(2) == 64)) && w.is_contiguous(), "w: [N, K] or [K / 64, N, 64]");
  const int M = x.size(0), N = panel ? w.size(1) : w.size(0), K = panel ? w.size(0) * 64 : w.size(1);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && x.size(1) == K, "x [M, K], 16-B rows");
  TORCH_CHECK(M >= 1 && M <= 16 && K % 64 == 0, "M in [1, 16], K % 64 == 0");
  TORCH_CHECK(ntw == 1 || ntw == 2, "ntw 1 or 2");
  TORCH_CHECK(epi >= 0 && epi <= 3 && (epi < 2 || ntw == 2), "epi 0-3; QKV / SwiGLU need ntw 2");
  const int nc = 16 * (int)ntw, tiles = (N + nc - 1) / nc;
  int kchunk = (K + (int)splits - 1) / (int)splits;
  kchunk = (kchunk + 31) & ~31;
  const int S = (K + kchunk - 1) / kchunk;
  if (S > 1) {
    TORCH_CHECK(part.numel() >= (int64_t)S * tiles * nc * 16, "split-K workspace too small");
    TORCH_CHECK(counters.numel() >= tiles, "counter buffer too small");
  }
  void* yp = nullptr;
  long ldy = 0;
  if (epi == 0 || epi == 3) {
    TORCH_CHECK(y.has_value(), "y required");
    check_bf16(*y, "y");
    TORCH_CHECK(y->dim() == 2 && y->stride(1) == 1 && y->size(0) == M && y->size(1) == (epi == 3 ? N / 2 : N), "y shape");
    yp = y->data_ptr();
    ldy = y->stride(0);
  }
  void* rp = nullptr;
  long ldr = 0;
  float* so = nullptr;
  long so_ld = 0;
  if (epi == 1) {
    TORCH_CHECK(res.has_value() && ssq_out.has_value(), "residual epilogue: res and ssq_out");
    check_bf16(*res, "res");
    check_f32(*ssq_out, "ssq_out");
    TORCH_CHECK(res->dim() == 2 && res->stride(1) == 1 && res->size(0) == M && res->size(1) == N, "res [M, N]");
    TORCH_CHECK(ssq_out->dim() == 2 && ssq_out->size(0) >= tiles && ssq_out->size(1) >= M, "ssq_out [>= tiles, >= M]");
    rp = res->data_ptr();
    ldr = res->stride(0);
    so = ssq_out->data_ptr<float>();
    so_ld = ssq_out->size(1);
  }
  const float* si = nullptr;
  long si_ld = 0;
  if (epi >= 2) {
    TORCH_CHECK(ssq_in.has_value(), "row-scaled epilogue: ssq_in");
    check_f32(*ssq_in, "ssq_in");
    TORCH_CHECK(ssq_in->dim() == 2 && ssq_in->size(1) >= M && ssq_n >= 1 && ssq_n <= ssq_in->size(0), "ssq_in [slots, >= M]");
    si = ssq_in->data_ptr<float>();
    si_ld = ssq_in->size(1);
  }
  const int *pp = nullptr, *sl = nullptr;
  const float* cs = nullptr;
  void *qo = nullptr, *kp = nullptr, *vp = nullptr;
  if (epi == 2) {
    TORCH_CHECK(pos.has_value() && cos_sin.has_value() && slots.has_value() && q_out.has_value() && kc.has_value() &&
                    vc.has_value(), "qkv epilogue operands");
    check_i32(*pos, "positions");
    check_i32(*slots, "slots");
    check_f32(*cos_sin, "cos_sin");
    check_bf16(*q_out, "q_out");
    check_bf16(*kc, "k_cache");
    check_bf16(*vc, "v_cache");
    TORCH_CHECK(d % 32 == 0 && N == (nq + 2 * nkv) * d, "qkv: N == (nq + 2 nkv) d, d % 32 == 0");
    TORCH_CHECK(pos->numel() >= M && slots->numel() >= M && cos_sin->dim() == 2 && cos_sin->size(1) == d,
                "positions / slots / cos_sin");
    TORCH_CHECK(q_out->is_contiguous() && q_out->numel() >= (int64_t)M * nq * d, "q_out [M, nq, d]");
    TORCH_CHECK(kc->is_contiguous() && vc->is_contiguous() && kc->dim() == 4 && kc->size(1) == nkv &&
                    kc->size(2) == 16 && kc->size(3) == d && vc->size(1) == nkv && vc->size(2) == d && vc->size(3) == 16,
                "cache layout: K [blocks, nkv, 16, d], V [blocks, nkv, d, 16]");
    pp = pos->data_ptr<int>();
    sl = slots->data_ptr<int>();
    cs = cos_sin->data_ptr<float>();
    qo = q_out->data_ptr();
    kp = kc->data_ptr();
    vp = vc->data_ptr();
  }
  ok(dllm_skinny_epi(x.data_ptr(), x.stride(0), w.data_ptr(), panel ? 1 : 0, yp, ldy, M, N, K, (int)ntw, (int)splits,
                     (int)epi, part.data_ptr<float>(), counters.data_ptr<int>(), rp, ldr, so, so_ld, si, (int)ssq_n, si_ld,
                     (float)scale, (float)eps, pp, cs, sl, qo, kp, vp, (int)nq, (int)nkv, (int)d, stream()),
     "skinny_epi");
  return epi == 1 ? tiles : 0;
}

// Small-batch GEMV (M in {1, 2, 4, 8}; csrc/kernels/gemv.hip): y = x . w^T (x = silu(g)*u if swiglu).
void gemv(torch::Tensor x, torch::Tensor w, torch::Tensor y, int64_t R, bool swiglu) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_bf16(y, "y");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && w.dim() == 2 && w.is_contiguous() && y.dim() == 2 &&
                  y.stride(1) == 1,
              "2-D row-major operands");
  const int M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(M == 1 || M == 2 || M == 4 || M == 8, "gemv: M in {1, 2, 4, 8}");
  TORCH_CHECK(x.size(1) == (swiglu ? 2 * K : K) && K % 8 == 0, "gemv: x inner dim, K % 8 == 0");
  TORCH_CHECK((int64_t)M * K * 2 <= 64 * 1024, "gemv: M x K bf16 must fit the 64 KB LDS stage");
  TORCH_CHECK(x.stride(0) % 8 == 0 && y.stride(0) >= N && y.size(0) == M && y.size(1) == N, "gemv: y shape / alignment");
  TORCH_CHECK(R == 1 || R == 2 || R == 4, "gemv: R in {1, 2, 4}");
  ok(dllm_gemv(x.data_ptr(), x.stride(0), w.data_ptr(), y.data_ptr(), y.stride(0), M, N, K, (int)R, swiglu ? 1 : 0,
               nullptr, nullptr, nullptr, 0.f, stream()),
     "gemv");
}

// RMSNorm-fused GEMV: r = x + res_in -> res_out (bf16), y = rmsnorm(r) * norm_w . w^T
void gemv_norm(torch::Tensor x, torch::Tensor res_in, torch::Tensor res_out, torch::Tensor norm_w, double eps,
               torch::Tensor w, torch::Tensor y, int64_t R) {
  for (auto* t : {&x, &res_in, &res_out, &norm_w, &w, &y}) check_bf16(*t, "gemv_norm operand");
  const int M = x.size(0), N = w.size(0), K = w.size(1);
  TORCH_CHECK(M == 1 || M == 2 || M == 4 || M == 8, "gemv_norm: M in {1, 2, 4, 8}");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(1) == K && K % 8 == 0, "gemv_norm: x [M, K]");
  TORCH_CHECK(res_in.is_contiguous() && res_out.is_contiguous() && res_in.sizes() == x.sizes() &&
                  res_out.sizes() == x.sizes() && res_in.data_ptr() != res_out.data_ptr(),
              "gemv_norm: res_in/res_out [M, K], distinct");
  TORCH_CHECK(norm_w.numel() == K && w.is_contiguous() && y.dim() == 2 && y.size(0) == M && y.size(1) == N &&
                  y.stride(1) == 1,
              "gemv_norm: shapes");
  TORCH_CHECK((int64_t)M * K * 2 <= 64 * 1024 && (R == 1 || R == 2 || R == 4), "gemv_norm: LDS stage / R");
  ok(dllm_gemv(x.data_ptr(), K, w.data_ptr(), y.data_ptr(), y.stride(0), M, N, K, (int)R, 0, res_in.data_ptr(),
               res_out.data_ptr(), norm_w.data_ptr(), (float)eps, stream()),
     "gemv_norm");
}

// GEMV with a fused decoder-layer epilogue (csrc/kernels/gemv.hip EPI; batch <= 8):
//   gemv_resadd: r += x . w^T in place, partial row sums of r^2 -> ssq_out [slots, >= M]; returns slots
//   gemv_qkv   : q [M, nq, d] of rope(rinv * x . w^T), K / V^T into the paged caches
//   gemv_swiglu: act [M, N/2] = silu(g) * u of rinv * x . w^T (interleaved gate/up rows)
static void gemv_epi_checks(const torch::Tensor& x, const torch::Tensor& w, int64_t R, const char* what) {
  check_bf16(x, what);
  check_bf16(w, what);
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && w.dim() == 2 && w.is_contiguous(), what, ": 2-D row-major operands");
  const int64_t M = x.size(0), K = w.size(1);
  TORCH_CHECK(M == 1 || M == 2 || M == 4 || M == 8, what, ": M in {1, 2, 4, 8}");
  TORCH_CHECK(x.size(1) == K && K % 8 == 0 && x.stride(0) % 8 == 0, what, ": x [M, K], K % 8 == 0, aligned rows");
  TORCH_CHECK(M * K * 2 <= 64 * 1024 && (R == 1 || R == 2 || R == 4), what, ": LDS stage / R");
}

static void check_ssq_in(const torch::Tensor& ssq, int64_t ssq_n, int64_t M) {
  check_f32(ssq, "ssq");
  TORCH_CHECK(ssq.dim() == 2 && ssq.stride(1) == 1 && ssq.size(1) >= M && ssq_n >= 1 && ssq_n <= ssq.size(0),
              "ssq [slots, >= M]");
}

int64_t gemv_slots(int64_t M, int64_t N, int64_t R) { return dllm_gemv_slots((int)M, (int)N, (int)R); }
void gemv_set_grid(int64_t min_blocks, int64_t xdiv, int64_t n_min) {
  dllm_gemv_set_grid((int)min_blocks, (int)xdiv, (int)n_min);
}

int64_t gemv_resadd(torch::Tensor x, torch::Tensor w, torch::Tensor r, torch::Tensor ssq_out, int64_t R) {
  gemv_epi_checks(x, w, R, "gemv_resadd");
  check_bf16(r, "r");
  check_f32(ssq_out, "ssq_out");
  const int M = x.size(0), N = w.size(0), K = w.size(1);
  const int slots = dllm_gemv_slots(M, N, (int)R);
  TORCH_CHECK(r.dim() == 2 && r.stride(1) == 1 && r.size(0) == M && r.size(1) == N && r.stride(0) % 8 == 0, "r [M, N]");
  TORCH_CHECK(ssq_out.dim() == 2 && ssq_out.stride(1) == 1 && ssq_out.size(0) >= slots && ssq_out.size(1) >= M,
              "ssq_out [>= slots, >= M]");
  ok(dllm_gemv_epi(x.data_ptr(), x.stride(0), w.data_ptr(), nullptr, 0, M, N, K, (int)R, 1, r.data_ptr(), r.stride(0),
                   ssq_out.data_ptr<float>(), ssq_out.stride(0), nullptr, 0, 0, 0.f, 0.f, nullptr, nullptr, nullptr,
                   nullptr, nullptr, nullptr, 0, 0, 0, stream()),
     "gemv_resadd");
  return slots;
}

void gemv_qkv(torch::Tensor x, torch::Tensor w, torch::Tensor ssq, int64_t ssq_n, double scale, double eps,
              torch::Tensor pos, torch::Tensor cos_sin, torch::Tensor slots, torch::Tensor q_out, torch::Tensor kc,
              torch::Tensor vc, int64_t nq, int64_t nkv, int64_t d, int64_t R) {
  gemv_epi_checks(x, w, R, "gemv_qkv");
  const int M = x.size(0), N = w.size(0), K = w.size(1);
  check_ssq_in(ssq, ssq_n, M);
  check_i32(pos, "positions");
  check_i32(slots, "slots");
  check_f32(cos_sin, "cos_sin");
  for (auto* t : {&q_out, &kc, &vc}) check_bf16(*t, "qkv outputs");
  TORCH_CHECK(N == (nq + 2 * nkv) * d && d % 32 == 0, "gemv_qkv: w rows (nq + 2 nkv) d, d % 32 == 0");
  TORCH_CHECK(pos.numel() >= M && slots.numel() >= M && cos_sin.dim() == 2 && cos_sin.size(1) == d &&
                  cos_sin.is_contiguous(),
              "positions/slots/cos_sin");
  TORCH_CHECK(q_out.is_contiguous() && q_out.numel() >= (int64_t)M * nq * d, "q_out");
  TORCH_CHECK(kc.is_contiguous() && vc.is_contiguous() && kc.size(1) == nkv && kc.size(2) == 16 && kc.size(3) == d &&
                  vc.size(2) == d && vc.size(3) == 16,
              "cache layout");
  ok(dllm_gemv_epi(x.data_ptr(), x.stride(0), w.data_ptr(), nullptr, 0, M, N, K, (int)R, 2, nullptr, 0, nullptr, 0,
                   ssq.data_ptr<float>(), (int)ssq_n, ssq.stride(0), (float)scale, (float)eps, pos.data_ptr<int>(),
                   cos_sin.data_ptr<float>(), slots.data_ptr<int>(), q_out.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                   (int)nq, (int)nkv, (int)d, stream()),
     "gemv_qkv");
}

void gemv_swiglu(torch::Tensor x, torch::Tensor w, torch::Tensor ssq, int64_t ssq_n, double scale, double eps,
                 torch::Tensor act, int64_t R) {
  gemv_epi_checks(x, w, R, "gemv_swiglu");
  const int M = x.size(0), N = w.size(0), K = w.size(1);
  check_ssq_in(ssq, ssq_n, M);
  check_bf16(act, "act");
  TORCH_CHECK(N % 32 == 0 && act.dim() == 2 && act.stride(1) == 1 && act.size(0) == M && act.size(1) == N / 2,
              "gemv_swiglu: act [M, N/2], N % 32 == 0");
  ok(dllm_gemv_epi(x.data_ptr(), x.stride(0), w.data_ptr(), act.data_ptr(), act.stride(0), M, N, K, (int)R, 3, nullptr,
                   0, nullptr, 0, ssq.data_ptr<float>(), (int)ssq_n, ssq.stride(0), (float)scale, (float)eps, nullptr,
                   nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, stream()),
     "gemv_swiglu");
}

// Mixtral-style MoE FFN: x [T, H] bf16, ids [T, k] int32, wts [T, k] f32, w13 [E, 2I, H], w2 [E, H, I]
// -> out [T, H] bf16 (partial sum over this rank's I shard under TP).  Workspace from torch's
// caching allocator, so the call is graph-capturable.
// grouped-tgemm MoE (csrc/kernels/moe.hip dllm_moe_ffn_tg): w13 interleaved per 16-row group
void moe_ffn_tg(torch::Tensor x, torch::Tensor ids, torch::Tensor wts, torch::Tensor w13, torch::Tensor w2,
                torch::Tensor out, std::vector<int64_t> plan) {
  check_bf16(x, "x");
  check_i32(ids, "ids");
  check_f32(wts, "wts");
  check_bf16(w13, "w13");
  check_bf16(w2, "w2");
  check_bf16(out, "out");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0 && out.is_contiguous(), "x rows 16-B aligned");
  TORCH_CHECK(w13.dim() == 3 && w2.dim() == 3 && w13.is_contiguous() && w2.is_contiguous(), "w13/w2 [E, N, K]");
  const int64_t T = x.size(0), H = x.size(1), E = w13.size(0), I = w13.size(1) / 2;
  TORCH_CHECK(w13.size(2) == H && w2.size(0) == E && w2.size(1) == H && w2.size(2) == I, "expert weight shapes");
  TORCH_CHECK(H % 64 == 0 && I % 64 == 0 && E <= 64, "H, I multiples of 64; E <= 64");
  TORCH_CHECK(ids.dim() == 2 && ids.size(0) == T && wts.sizes() == ids.sizes() && ids.is_contiguous() &&
                  wts.is_contiguous(), "ids/wts [T, k]");
  TORCH_CHECK(out.size(0) == T && out.size(1) == H, "out shape");
  TORCH_CHECK(plan.size() == 9, "plan: bm, bn13, stages13, ks13, nw13, bn2, stages2, ks2, nw2");
  const int bm = (int)plan[0];
  for (int g = 0; g < 2; ++g) {
    const int bn = (int)plan[1 + 4 * g], st = (int)plan[2 + 4 * g], ks = (int)plan[3 + 4 * g], nw = (int)plan[4 + 4 * g];
    TORCH_CHECK((ks == 1 || ks == 2) && (nw == 4 || (nw == 8 && bn >= 128)) &&
                    (st == 2 || st == 3 || ((st == 4 || st == 6) && ks == 1 && bm <= 128)) &&
                    (bm == 64 || bm == 128 || ((bm == 192 || bm == 256) && nw == 8)) &&
                    (bn == 64 || bn == 128 || (bn == 256 && bm == 256)) && st * ks * (bm + bn) * 128 <= 150 * 1024,
                "moe plan tile / ring size");
    TORCH_CHECK((g == 0 ? H : I) % (64 * ks) == 0, "K % (64 ks)");
  }
  const int k = ids.size(1);
  auto iopt = ids.options();
  const int P = (int)(T * k), mt = dllm_moe_max_tiles_bm(P, (int)E, bm);
  auto perm = torch::empty({std::max(P, 1)}, iopt);
  auto inv = torch::empty({std::max(P, 1)}, iopt);
  auto tiles = torch::empty({4 * mt + 1}, iopt);
  auto act = torch::empty({std::max(P, 1), I}, x.options());
  auto y = torch::empty({std::max(P, 1), H}, x.options());
  int pl[9];
  for (int i = 0; i < 9; ++i) pl[i] = (int)plan[i];
  ok(dllm_moe_ffn_tg(x.data_ptr(), x.stride(0), T, (int)H, ids.data_ptr<int>(), wts.data_ptr<float>(), k, (int)E,
                     w13.data_ptr(), w2.data_ptr(), (int)I, perm.data_ptr<int>(), inv.data_ptr<int>(),
                     tiles.data_ptr<int>(), act.data_ptr(), y.data_ptr(), out.data_ptr(), pl, stream()),
     "moe_ffn_tg");
}

void moe_ffn(torch::Tensor x, torch::Tensor ids, torch::Tensor wts, torch::Tensor w13, torch::Tensor w2,
             torch::Tensor out) {
  check_bf16(x, "x");
  check_i32(ids, "ids");
  check_f32(wts, "wts");
  check_bf16(w13, "w13");
  check_bf16(w2, "w2");
  check_bf16(out, "out");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && out.is_contiguous(), "x 2-D row-major, out contiguous");
  TORCH_CHECK(w13.dim() == 3 && w2.dim() == 3 && w13.is_contiguous() && w2.is_contiguous(), "w13/w2 [E, N, K]");
  const int64_t T = x.size(0), H = x.size(1), E = w13.size(0), I = w13.size(1) / 2;
  TORCH_CHECK(w13.size(2) == H && w2.size(0) == E && w2.size(1) == H && w2.size(2) == I, "expert weight shapes");
  TORCH_CHECK(ids.dim() == 2 && ids.size(0) == T && wts.sizes() == ids.sizes(), "ids/wts [T, k]");
  TORCH_CHECK(out.size(0) == T && out.size(1) == H, "out shape");
  const int k = ids.size(1);
  auto iopt = ids.options();
  const int P = (int)(T * k), mt = dllm_moe_max_tiles(P, (int)E);
  auto perm = torch::empty({std::max(P, 1)}, iopt);
  auto tiles = torch::empty({4 * mt}, iopt);
  auto act = torch::empty({std::max(P, 1), I}, x.options());
  auto y = torch::empty({std::max(P, 1), H}, wts.options());
  ok(dllm_moe_ffn(x.data_ptr(), x.stride(0), T, (int)H, ids.data_ptr<int>(), wts.data_ptr<float>(), k, (int)E,
                  w13.data_ptr(), w2.data_ptr(), (int)I, perm.data_ptr<int>(), tiles.data_ptr<int>(), act.data_ptr(),
                  y.data_ptr<float>(), out.data_ptr(), stream()),
     "moe_ffn");
}

// ---- one-shot all-reduce over IPC-mapped peer buffers (csrc/kernels/custom_ar.hip)
int64_t car_alloc(int64_t data_bytes) {
  void* p = nullptr;
  ok(dllm_car_alloc(data_bytes, &p), "car_alloc");
  return (int64_t)p;
}
py::bytes car_handle(int64_t base) {
  char buf[64] = {0};
  ok(dllm_car_get_handle((void*)base, buf), "hipIpcGetMemHandle");
  return py::bytes(buf, dllm_car_handle_size());
}
int64_t car_open(py::bytes h) {
  std::string s = h;
  TORCH_CHECK((int)s.size() == dllm_car_handle_size(), "bad IPC handle size");
  void* p = nullptr;
  ok(dllm_car_open_handle(s.data(), &p), "hipIpcOpenMemHandle");
  return (int64_t)p;
}
void car_close(int64_t base) { ok(dllm_car_close_handle((void*)base), "hipIpcCloseMemHandle"); }
void car_free(int64_t base) { ok(dllm_car_free((void*)base), "hipFree"); }
void car_allreduce(torch::Tensor x, torch::Tensor out, std::vector<int64_t> bases, int64_t rank, int64_t data_bytes,
                   torch::Tensor counters, torch::Tensor err, int64_t spin_limit) {
  check_bf16(x, "x");
  check_bf16(out, "out");
  check_i32(counters, "counters");
  check_i32(err, "err");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.numel() == out.numel(), "contiguous, same size");
  TORCH_CHECK(counters.numel() >= 2 && err.numel() >= 1, "counters[2], err[1]");
  const int64_t nbytes = x.numel() * 2;
  TORCH_CHECK(nbytes % 16 == 0 && nbytes <= data_bytes, "message must be a multiple of 16 B and fit the buffer");
  TORCH_CHECK(!bases.empty() && bases.size() <= 8 && rank >= 0 && rank < (int64_t)bases.size(), "bad ranks");
  void* b[8];
  for (size_t i = 0; i < bases.size(); ++i) b[i] = (void*)bases[i];
  ok(dllm_car_allreduce(x.data_ptr(), out.data_ptr(), nbytes, b, (int)bases.size(), (int)rank, data_bytes,
                        (unsigned*)counters.data_ptr<int>(), err.data_ptr<int>(), spin_limit, stream()),
     "car_allreduce");
}

// r = bf16(sum_p y_p) + r (add) or r = bf16(sum_p y_p), in place, and the new r's partial row sums
// of squares per column slice into ssq [slots, >= T]; returns the slot count (one-shot all-reduce
// with the fused residual / RMSNorm-statistics epilogue, csrc/kernels/custom_ar.hip)
int64_t car_resadd(torch::Tensor y, torch::Tensor r, torch::Tensor ssq, bool add, std::vector<int64_t> bases,
                   int64_t rank, int64_t data_bytes, torch::Tensor counters, torch::Tensor err, int64_t spin_limit) {
  check_bf16(y, "y");
  check_bf16(r, "r");
  check_f32(ssq, "ssq");
  check_i32(counters, "counters");
  check_i32(err, "err");
  TORCH_CHECK(y.dim() == 2 && y.is_contiguous() && r.dim() == 2 && r.stride(1) == 1 && r.sizes() == y.sizes(),
              "y [T, H] contiguous, r like y (row stride may differ)");
  const int H = (int)y.size(1), T = (int)y.size(0);
  const int slots = dllm_car_resadd_slots(H);
  TORCH_CHECK(slots >= 1, "hidden size has no column-slice split");
  TORCH_CHECK(ssq.dim() == 2 && ssq.size(0) >= slots && ssq.size(1) >= T && ssq.stride(1) == 1, "ssq [>= slots, >= T]");
  TORCH_CHECK((int64_t)T * H * 2 <= data_bytes, "message must fit the buffer");
  TORCH_CHECK(!bases.empty() && bases.size() <= 8 && rank >= 0 && rank < (int64_t)bases.size(), "bad ranks");
  void* b[8];
  for (size_t i = 0; i < bases.size(); ++i) b[i] = (void*)bases[i];
  const int n = dllm_car_resadd(y.data_ptr(), r.data_ptr(), r.stride(0), ssq.data_ptr<float>(), ssq.stride(0), T, H,
                                add ? 1 : 0, b, (int)bases.size(), (int)rank, data_bytes,
                                (unsigned*)counters.data_ptr<int>(), err.data_ptr<int>(), spin_limit, stream());
  TORCH_CHECK(n >= 1, "car_resadd failed (", n, ")");
  return n;
}
int64_t car_resadd_slots(int64_t H) { return dllm_car_resadd_slots((int)H); }
void car_allgather(torch::Tensor x, torch::Tensor out, std::vector<int64_t> bases, int64_t rank, int64_t data_bytes,
                   torch::Tensor counters, torch::Tensor err, int64_t spin_limit) {
  check_i32(counters, "counters");
  check_i32(err, "err");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.scalar_type() == out.scalar_type(), "contiguous, same dtype");
  TORCH_CHECK(out.numel() == x.numel() * (int64_t)bases.size(), "out = world x input");
  const int64_t nbytes = x.numel() * x.element_size();
  TORCH_CHECK(nbytes % 16 == 0 && nbytes <= data_bytes, "message must be a multiple of 16 B and fit the buffer");
  TORCH_CHECK(!bases.empty() && bases.size() <= 8 && rank >= 0 && rank < (int64_t)bases.size(), "bad ranks");
  void* b[8];
  for (size_t i = 0; i < bases.size(); ++i) b[i] = (void*)bases[i];
  ok(dllm_car_allgather(x.data_ptr(), out.data_ptr(), nbytes, b, (int)bases.size(), (int)rank, data_bytes,
                        (unsigned*)counters.data_ptr<int>(), err.data_ptr<int>(), spin_limit, stream()),
     "car_allgather");
}
// In-graph health vote glue around the 16-byte one-shot all-reduce (mode 0: stage, 1: decide).
void car_vote(int64_t mode, torch::Tensor err, torch::Tensor v, torch::Tensor out) {
  check_i32(err, "err");
  check_i32(out, "out");
  TORCH_CHECK(v.scalar_type() == torch::kBFloat16 && v.numel() >= 8 && v.is_contiguous(), "car_vote: v bf16 [>= 8]");
  TORCH_CHECK(err.numel() >= 2 && out.numel() >= 1, "car_vote: err [flag, staged snapshot] / out");
  ok(dllm_car_vote((int)mode, err.data_ptr<int>(), v.data_ptr(), out.data_ptr<int>(), stream()), "car_vote");
}

// ---- fused-epilogue LDS-tiled GEMM (csrc/kernels/tgemm.hip).  epi: 0 plain y = x.w^T (optionally
// row-scaled by rinv from ssq_in), 1 residual add (y = residual, in place; ssq_out partial row
// sums), 2 QKV (RoPE + q_out + paged K/V writes), 3 SwiGLU (y = [M, N/2]), 4 GELU (y = gelu(x.w^T +
// bias)).  bias [N] (epi 0, 1, 4) is added to the product before the epilogue op.
void tgemm(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> y, int64_t epi, int64_t bm, int64_t bn,
           int64_t stages, int64_t splits, int64_t ks, int64_t nw, c10::optional<torch::Tensor> part, c10::optional<torch::Tensor> counters,
           c10::optional<torch::Tensor> ssq_in, int64_t ssq_in_n, double norm_scale, double eps,
           c10::optional<torch::Tensor> ssq_out, c10::optional<torch::Tensor> pos,
           c10::optional<torch::Tensor> cos_sin, c10::optional<torch::Tensor> slots,
           c10::optional<torch::Tensor> q_out, c10::optional<torch::Tensor> kc, c10::optional<torch::Tensor> vc,
           int64_t nq, int64_t nkv, int64_t d, c10::optional<torch::Tensor> bias, int64_t wk, int64_t nl,
           c10::optional<torch::Tensor> sk_table, int64_t sk_cmax, c10::optional<torch::Tensor> v_rows,
           int64_t kdepth, int64_t mfma, int64_t raster) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  TORCH_CHECK(mfma == 16 || mfma == 32, "tgemm: mfma 16 or 32");
  if (mfma == 32) {   // tgemm.hip by_tile_m32 minus kPruned: the whitelist, so a bad plan gets a clear error
    const bool known = wk == 1 && kdepth == 64 &&
                       ((nl == 0 && ks == 2 && stages == 3 && ((bm == 64 && bn == 64 && nw == 4) ||
                                                               (bm == 64 && bn == 128 && nw == 8))));
    TORCH_CHECK(known, "tgemm: no 32x32x16 plan (", bm, "x", bn, ", ", stages, " stages, ks ", ks, ", ", nw, "+", nl,
                " waves)");
    TORCH_CHECK(!sk_table.has_value(), "tgemm: 32x32x16 plans have no stream-K form");
  }
  if (kdepth == 32) {   // tgemm.hip by_tile_k32 minus kPruned: explicit whitelist
    const bool known = ks == 1 && wk == 1 && nw == 8 && bm == 256 && bn == 256 && stages == 4 && nl == 0;
    TORCH_CHECK(known, "tgemm: no 32-deep plan (", bm, "x", bn, ", ", stages, " stages, ", nw, "+", nl, " waves)");
  }
  if (nl > 0 && kdepth != 32 && mfma == 16) {  // loader-wave plans (tgemm.hip by_tile_nl minus kPruned): KS 1, one k-group
    const bool known = ks == 1 && wk == 1 &&
                       ((bm == 16 && bn == 128 && nw == 4 && nl == 6 && (stages == 4 || stages == 8)) ||
                        (bm == 64 && bn == 64 && nw == 4 && ((nl == 4 && stages == 4) || (nl == 8 && (stages == 4 || stages == 8)))) ||
                        (bm == 128 && bn == 64 && nw == 4 && (nl == 4 || nl == 8) && stages == 4) ||
                        (bm == 128 && bn == 128 && nw == 4 && nl == 8 && stages == 4) ||
                        (bm == 160 && bn == 128 && nw == 8 && (nl == 4 || nl == 6) && stages == 3) ||
                        (bm == 256 && bn == 128 && nw == 8 && (nl == 4 || nl == 8) && stages == 3));
    TORCH_CHECK(known, "tgemm: no loader-wave plan (", bm, "x", bn, ", ", stages, " stages, ", nw, "+", nl, " waves)");
  }
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1 && x.stride(0) % 8 == 0, "x: 2-D row-major, 16-B aligned rows");
  TORCH_CHECK(epi >= 0 && epi <= 4, "epi");
  // w: [N, K] row-major, or the K-panel-major copy [K / 64, N, 64] (models.llama.panel_weight)
  const bool panel = w.dim() == 3;
  TORCH_CHECK(((w.dim() == 2) || (panel && w.size(2) == 64)) && w.is_contiguous(),
              "w: [N, K] or [K / 64, N, 64] contiguous");
  const int M = x.size(0), N = panel ? w.size(1) : w.size(0), K = panel ? w.size(0) * 64 : w.size(1);
  TORCH_CHECK((ks == 1 || ks == 2) && (nw == 4 || (nw == 8 && bn >= 128)), "ks in {1,2}; nw 4, or 8 with bn >= 128");
  TORCH_CHECK(wk == 1 || (wk == 2 && nw == 4 && ks == 2 && stages <= 3 && bm <= 128 && bn <= 128),
              "wk 2: two k-groups of 4 waves, ks 2, 2-3 stages, tiles up to 128 x 128");
  TORCH_CHECK(x.size(1) == K && K % (64 * ks) == 0, "x [M, K], K % (64 ks) == 0");
  TORCH_CHECK(nl > 0 || kdepth == 32 || ((bm == 64 || bm == 128 || ((bm == 192 || bm == 256) && nw == 8)) && (bn == 64 || bn == 128 || (bn == 256 && bm == 256)) &&
                  (stages == 2 || stages == 3 || ((stages == 4 || stages == 6) && ks == 1 && bm <= 128)) &&
                  (int64_t)stages * ks * (bm + bn) * 128 <= 150 * 1024),
              "tile / ring size");
  TORCH_CHECK(splits >= 1 && splits <= 64, "splits");
  const int kq = 64 * (int)ks;
  int kchunk = (K + splits - 1) / splits;
  kchunk = (kchunk + kq - 1) / kq * kq;
  const int S = (K + kchunk - 1) / kchunk;
  const int64_t tiles = (int64_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  dllm::GemmArgs a{};
  a.A = (const uint16_t*)x.data_ptr();
  a.lda = x.stride(0);
  a.W = (const uint16_t*)w.data_ptr();
  a.M = M; a.N = N; a.K = K; a.kchunk = kchunk; a.splits = S;
  a.w_panel = panel ? 1 : 0;
  if (sk_table.has_value()) {   // stream-K: the host-built segment lists (ops.gemm.stream_k_table)
    check_i32(*sk_table, "sk_table");
    TORCH_CHECK(sk_table->dim() == 3 && sk_table->size(2) == 4 && sk_table->is_contiguous() &&
                    sk_table->size(0) >= 1 && sk_table->size(1) >= 1 && sk_cmax >= 1 && splits == 1,
                "sk_table [grid, segments, 4] int32, splits 1");
    TORCH_CHECK(part.has_value() && counters.has_value(), "stream-K needs part/counters workspaces");
    check_f32(*part, "part");
    check_i32(*counters, "counters");
    TORCH_CHECK(part->numel() >= sk_cmax * tiles * bm * bn && counters->numel() >= tiles,
                "stream-K workspace too small");
    a.part = part->data_ptr<float>();
    a.counters = counters->data_ptr<int>();
    a.sk_table = sk_table->data_ptr<int>();
    a.sk_grid = (int)sk_table->size(0);
    a.sk_segmax = (int)sk_table->size(1);
    a.sk_cmax = (int)sk_cmax;
  } else if (S > 1) {
    TORCH_CHECK(part.has_value() && counters.has_value(), "split-K needs part/counters workspaces");
    check_f32(*part, "part");
    check_i32(*counters, "counters");
    TORCH_CHECK(part->numel() >= (int64_t)S * tiles * bm * bn && counters->numel() >= tiles,
                "split-K workspace too small");
    a.part = part->data_ptr<float>();
    a.counters = counters->data_ptr<int>();
  }
  if (ssq_in.has_value()) {
    check_f32(*ssq_in, "ssq_in");
    TORCH_CHECK(ssq_in->dim() == 2 && ssq_in->size(1) >= M && ssq_in_n >= 1 && ssq_in_n <= ssq_in->size(0),
                "ssq_in [slots, >= M]");
    TORCH_CHECK(epi != 1, "residual epilogue takes no row scale");
    a.ssq_in = ssq_in->data_ptr<float>();
    a.ssq_in_n = ssq_in_n;
    a.ssq_in_ld = ssq_in->size(1);
    a.norm_scale = (float)norm_scale;
    a.eps = (float)eps;
  }
  if (bias.has_value()) {
    check_bf16(*bias, "bias");
    TORCH_CHECK(epi == 0 || epi == 1 || epi == 4, "bias: plain, residual or gelu epilogue");
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == N, "bias [N]");
    a.bias = (const uint16_t*)bias->data_ptr();
  }
  if (epi == 0 || epi == 1 || epi == 3 || epi == 4) {
    TORCH_CHECK(y.has_value(), "y required");
    check_bf16(*y, "y");
    TORCH_CHECK(y->dim() == 2 && y->stride(1) == 1 && y->size(0) == M && y->size(1) == (epi == 3 ? N / 2 : N),
                "y shape");
    a.Y = (uint16_t*)y->data_ptr();
    a.ldy = y->stride(0);
  }
  if (epi == 1 && ssq_out.has_value()) {
    check_f32(*ssq_out, "ssq_out");
    TORCH_CHECK(ssq_out->dim() == 2 && ssq_out->size(0) >= (N + bn - 1) / bn && ssq_out->size(1) >= M,
                "ssq_out [>= n_tiles, >= M]");
    a.ssq_out = ssq_out->data_ptr<float>();
    a.ssq_out_ld = ssq_out->size(1);
  }
  if (epi == 3) TORCH_CHECK(N % 32 == 0, "swiglu: N % 32 == 0");
  if (epi == 2) {
    TORCH_CHECK(pos.has_value() && cos_sin.has_value() && slots.has_value() && q_out.has_value() && kc.has_value() &&
                    vc.has_value(),
                "qkv epilogue operands");
    check_i32(*pos, "positions");
    check_i32(*slots, "slots");
    check_f32(*cos_sin, "cos_sin");
    check_bf16(*q_out, "q_out");
    check_bf16(*kc, "k_cache");
    check_bf16(*vc, "v_cache");
    TORCH_CHECK(d % 32 == 0 && N == (nq + 2 * nkv) * d, "qkv: N == (nq + 2 nkv) d, d % 32 == 0");
    TORCH_CHECK(pos->numel() >= M && slots->numel() >= M, "positions/slots length");
    TORCH_CHECK(cos_sin->dim() == 2 && cos_sin->size(1) == d, "cos_sin [max_pos, d]");
    TORCH_CHECK(q_out->is_contiguous() && q_out->numel() >= (int64_t)M * nq * d, "q_out [M, nq, d]");
    TORCH_CHECK(kc->is_contiguous() && vc->is_contiguous() && kc->dim() == 4 && kc->size(1) == nkv &&
                    kc->size(2) == 16 && kc->size(3) == d && vc->size(1) == nkv && vc->size(2) == d &&
                    vc->size(3) == 16,
                "cache layout: K [blocks, nkv, 16, d], V [blocks, nkv, d, 16]");
    a.pos = pos->data_ptr<int>();
    a.cos_sin = cos_sin->data_ptr<float>();
    a.slots = slots->data_ptr<int>();
    a.q_out = (uint16_t*)q_out->data_ptr();
    a.kc = (uint16_t*)kc->data_ptr();
    a.vc = (uint16_t*)vc->data_ptr();
    a.nq = nq; a.nkv = nkv; a.d = d;
    if (v_rows.has_value()) {   // V row-major [M, nkv * d] instead of the V^T cache (decode attention writes it)
      check_bf16(*v_rows, "v_rows");
      TORCH_CHECK(v_rows->dim() == 2 && v_rows->stride(1) == 1 && v_rows->size(0) >= M && v_rows->size(1) == nkv * d &&
                      v_rows->stride(0) % 8 == 0,
                  "v_rows [>= M, nkv * d], 16-B aligned rows");
      a.v_rows = (uint16_t*)v_rows->data_ptr();
      a.v_ld = v_rows->stride(0);
    }
  }
  TORCH_CHECK(kdepth == 64 || kdepth == 32, "tgemm: k depth 64 or 32");
  a.kdepth = (int)kdepth;
  a.mfma = (int)mfma;
  TORCH_CHECK(raster >= 0 && raster <= 64, "tgemm: raster 0..64");
  a.raster = (int)raster;
  ok(dllm_tgemm(&a, (int)bm, (int)bn, (int)stages, (int)ks, (int)nw, (int)wk, (int)epi, stream(), (int)nl), "tgemm");
}

// standalone EPI_QKV / EPI_SWIGLU for a vendor-GEMM output y (prefill)
void qkv_post(torch::Tensor y, torch::Tensor ssq, int64_t ssq_n, double scale, double eps, torch::Tensor pos,
              torch::Tensor cos_sin, torch::Tensor slots, torch::Tensor q_out, torch::Tensor kc, torch::Tensor vc,
              int64_t nq, int64_t nkv, int64_t d, c10::optional<torch::Tensor> v_rows) {
  check_bf16(y, "y");
  check_f32(ssq, "ssq");
  check_i32(pos, "positions");
  check_i32(slots, "slots");
  check_f32(cos_sin, "cos_sin");
  for (auto* t : {&q_out, &kc, &vc}) check_bf16(*t, "qkv outputs");
  const int M = y.size(0);
  TORCH_CHECK(y.dim() == 2 && y.stride(1) == 1 && y.size(1) == (nq + 2 * nkv) * d && d % 32 == 0, "y [M, (nq+2nkv) d]");
  TORCH_CHECK(ssq.dim() == 2 && ssq.size(1) >= M && ssq_n >= 1 && ssq_n <= ssq.size(0), "ssq [slots, >= M]");
  TORCH_CHECK(pos.numel() >= M && slots.numel() >= M && cos_sin.size(1) == d, "positions/slots/cos_sin");
  TORCH_CHECK(q_out.is_contiguous() && q_out.numel() >= (int64_t)M * nq * d, "q_out");
  TORCH_CHECK(kc.is_contiguous() && vc.is_contiguous() && kc.size(1) == nkv && kc.size(2) == 16 && kc.size(3) == d &&
                  vc.size(2) == d && vc.size(3) == 16,
              "cache layout");
  void* vr = nullptr;
  if (v_rows.has_value() && v_rows->defined()) {   // decode: V row-major, the attention kernel writes V^T
    check_bf16(*v_rows, "v_rows");
    TORCH_CHECK(v_rows->is_contiguous() && v_rows->numel() >= (int64_t)M * nkv * d, "v_rows [M, nkv d]");
    vr = v_rows->data_ptr();
  }
  ok(dllm_qkv_post(y.data_ptr(), y.stride(0), ssq.data_ptr<float>(), ssq_n, ssq.size(1), (float)scale, (float)eps,
                   pos.data_ptr<int>(), cos_sin.data_ptr<float>(), slots.data_ptr<int>(), q_out.data_ptr(), kc.data_ptr(),
                   vc.data_ptr(), vr, M, nq, nkv, d, stream()),
     "qkv_post");
}

void swiglu_post(torch::Tensor y, torch::Tensor ssq, int64_t ssq_n, double scale, double eps, torch::Tensor act) {
  check_bf16(y, "y");
  check_f32(ssq, "ssq");
  check_bf16(act, "act");
  const int M = y.size(0), N = y.size(1);
  TORCH_CHECK(y.dim() == 2 && y.stride(1) == 1 && N % 32 == 0, "y [M, 2I]");
  TORCH_CHECK(act.dim() == 2 && act.stride(1) == 1 && act.size(0) == M && act.size(1) == N / 2, "act [M, I]");
  TORCH_CHECK(ssq.dim() == 2 && ssq.size(1) >= M && ssq_n >= 1 && ssq_n <= ssq.size(0), "ssq [slots, >= M]");
  ok(dllm_swiglu_post(y.data_ptr(), y.stride(0), ssq.data_ptr<float>(), ssq_n, ssq.size(1), (float)scale, (float)eps,
                      act.data_ptr(), act.stride(0), M, N, stream()),
     "swiglu_post");
}

// r = h + r in place (h optional) and row sums of r^2: ssq f32 [M] (one slot) or [slots, >= M]
// (partial sums over up to ``slots`` column slices); returns the number of slots written
int64_t res_add_ssq(c10::optional<torch::Tensor> h, torch::Tensor r, torch::Tensor ssq) {
  check_bf16(r, "r");
  check_f32(ssq, "ssq");
  TORCH_CHECK(r.dim() == 2 && r.stride(1) == 1, "r [M, H]");
  TORCH_CHECK((ssq.dim() == 1 && ssq.numel() >= r.size(0)) ||
                  (ssq.dim() == 2 && ssq.size(1) >= r.size(0) && ssq.stride(1) == 1),
              "ssq [>= M] or [slots, >= M]");
  const void* hp = nullptr;
  long ldh = 0;
  if (h.has_value()) {
    check_bf16(*h, "h");
    TORCH_CHECK(h->dim() == 2 && h->stride(1) == 1 && h->sizes() == r.sizes(), "h like r");
    hp = h->data_ptr();
    ldh = h->stride(0);
  }
  const int slices = ssq.dim() == 2 ? (int)ssq.size(0) : 1;
  const long ld = ssq.dim() == 2 ? ssq.stride(0) : 0;
  const int n = dllm_res_add_ssq(hp, ldh, r.data_ptr(), r.stride(0), ssq.data_ptr<float>(), ld, slices, r.size(0),
                                 r.size(1), stream());
  TORCH_CHECK(n >= 1, "res_add_ssq failed (", n, ")");
  return n;
}


// router encoder (csrc/kernels/encoder.hip): bidirectional attention over a padded batch
void encoder_attention(torch::Tensor qkv, torch::Tensor lens, torch::Tensor out, int64_t B, int64_t S, int64_t nh,
                       int64_t d, double scale) {
  check_bf16(qkv, "qkv");
  check_bf16(out, "out");
  check_i32(lens, "lens");
  TORCH_CHECK(d == 32 || d == 64, "encoder attention: head_dim 32 or 64");
  TORCH_CHECK(S >= 1 && S <= 512, "encoder attention: 1 <= S <= 512");
  TORCH_CHECK(qkv.is_contiguous() && qkv.dim() == 2 && qkv.size(0) == B * S && qkv.size(1) == 3 * nh * d,
              "qkv [B*S, 3 nh d]");
  TORCH_CHECK(out.is_contiguous() && out.dim() == 2 && out.size(0) == B * S && out.size(1) == nh * d, "out [B*S, nh d]");
  TORCH_CHECK(lens.numel() >= B, "lens [B]");
  ok(dllm_encoder_attention(qkv.data_ptr(), lens.data_ptr<int>(), out.data_ptr(), B, S, nh, d, (float)scale, stream()),
     "encoder_attention");
}

void embed_ln(torch::Tensor ids, torch::Tensor word, torch::Tensor pos, torch::Tensor type0, torch::Tensor w,
              torch::Tensor b, torch::Tensor out, int64_t S, double eps) {
  check_i32(ids, "ids");
  for (auto* t : {&word, &pos, &type0, &w, &b, &out}) check_bf16(*t, "embed_ln operand");
  const int64_t T = ids.numel(), H = word.size(1);
  TORCH_CHECK(ids.is_contiguous() && word.is_contiguous() && pos.is_contiguous() && type0.is_contiguous() &&
                  w.is_contiguous() && b.is_contiguous() && out.is_contiguous(),
              "contiguous operands");
  TORCH_CHECK(S >= 1 && T % S == 0 && pos.size(0) >= S && pos.size(1) == H && type0.numel() == H && w.numel() == H &&
                  b.numel() == H && out.numel() == T * H && H % 8 == 0 && H <= 2048,
              "embed_ln shapes");
  ok(dllm_embed_ln(ids.data_ptr<int>(), word.data_ptr(), pos.data_ptr(), type0.data_ptr(), w.data_ptr(), b.data_ptr(),
                   out.data_ptr(), T, S, H, word.size(0), (float)eps, stream()),
     "embed_ln");
}
}  // namespace

PYBIND11_MODULE(_hip_kernels, m) {
  m.def("encoder_attention", &encoder_attention);
  m.def("embed_ln", &embed_ln);
  m.def("moe_ffn", &moe_ffn);
  m.def("moe_ffn_tg", &moe_ffn_tg);
  m.def("tgemm", &tgemm);
  m.def("res_add_ssq", &res_add_ssq);
  m.def("qkv_post", &qkv_post, py::arg("y"), py::arg("ssq"), py::arg("ssq_n"), py::arg("scale"), py::arg("eps"),
        py::arg("pos"), py::arg("cos_sin"), py::arg("slots"), py::arg("q_out"), py::arg("kc"), py::arg("vc"),
        py::arg("nq"), py::arg("nkv"), py::arg("d"), py::arg("v_rows") = py::none());
  m.def("swiglu_post", &swiglu_post);
  m.def("car_alloc", &car_alloc);
  m.def("car_handle", &car_handle);
  m.def("car_open", &car_open);
  m.def("car_close", &car_close);
  m.def("car_free", &car_free);
  m.def("car_allreduce", &car_allreduce);
  m.def("car_vote", &car_vote);
  m.def("car_resadd", &car_resadd);
  m.def("car_resadd_slots", &car_resadd_slots);
  m.def("car_allgather", &car_allgather);
  m.doc() = "gfx950 HIP kernels for distributed_llm_amd";
  m.def("norm", &norm);
  m.def("rope_kv", &rope_kv);
  m.def("kv_write", &kv_write);
  m.def("paged_attention", &paged_attention);
  m.def("flash_prefill", &flash_prefill, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("block_tables"),
        py::arg("qstart"), py::arg("qlen"), py::arg("ctx"), py::arg("tile_seq"), py::arg("tile_tok0"), py::arg("out"),
        py::arg("causal"), py::arg("scale"), py::arg("splits") = 1, py::arg("part_o") = py::none(),
        py::arg("part_ml") = py::none(), py::arg("counters") = py::none());
  m.def("silu_mul", &silu_mul);
  m.def("embed", &embed, py::arg("ids"), py::arg("table"), py::arg("out"), py::arg("lo"), py::arg("ssq") = py::none(),
        py::arg("sc_dst") = py::none(), py::arg("sc_buf") = py::none());
  m.def("gelu", &gelu);
  m.def("mean_pool_l2", &mean_pool_l2);
  m.def("moe_gate", &moe_gate);
  m.def("moe_router", &moe_router, py::arg("x"), py::arg("wg"), py::arg("k"), py::arg("ids"), py::arg("w"),
        py::arg("logits") = py::none());
  m.def("argmax", &argmax);
  m.def("scatter_pairs", &scatter_pairs);
  m.def("step_fetch", &step_fetch);
  m.def("step_store", &step_store);
  m.def("sample_topp", &sample_topp);
  m.def("sample_rows", &sample_rows);
  m.def("sample_split", &sample_split);
  m.def("sample_split_maxp", &sample_split_maxp);
  m.def("sample_split_kmax", &sample_split_kmax);
  m.def("tp_cands_k", &tp_cands_k);
  m.def("tp_cands", &tp_cands);
  m.def("tp_sample", &tp_sample);
  m.def("cosine_scores", &cosine_scores);
  m.def("cache_scan", &cache_scan);
  m.def("cache_write", &cache_write);
  m.def("skinny_gemm", &skinny_gemm);
  m.def("skinny_epi", &skinny_epi);
  m.def("gemv", &gemv);
  m.def("gemv_norm", &gemv_norm);
  m.def("gemv_slots", &gemv_slots);
  m.def("gemv_set_grid", &gemv_set_grid);
  m.def("gemv_resadd", &gemv_resadd);
  m.def("gemv_qkv", &gemv_qkv);
  m.def("gemv_swiglu", &gemv_swiglu);
}
