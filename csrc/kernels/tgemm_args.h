// Argument block of the fused-epilogue GEMM (csrc/kernels/tgemm.hip), shared with the host
// bindings (csrc/bindings.cpp) so both sides agree on the layout.
#pragma once
#include <stdint.h>

namespace dllm {
struct GemmArgs {
  const uint16_t* A;
  long lda;
  const uint16_t* W;  // [N, K] contiguous
  uint16_t* Y;        // PLAIN [M, N]; RESADD residual [M, N] (in place); SWIGLU [M, N / 2]; QKV unused
  long ldy;
  int M, N, K;
  int kchunk, splits;
  float* part;    // split-K slabs
  int* counters;  // split-K tickets, one per output tile (zeroed; re-armed by the last arriver)
  // row scale rinv[m] = rsqrt(sum_s ssq_in[s * ssq_in_ld + m] * norm_scale + eps)  (null: none)
  const float* ssq_in;
  int ssq_in_n;
  long ssq_in_ld;
  float norm_scale, eps;
  // RESADD: partial row sums of squares ssq_out[n_tile * ssq_out_ld + m]
  float* ssq_out;
  long ssq_out_ld;
  // QKV
  const int* pos;
  const float* cos_sin;  // [max_pos, d]: cos in [:d/2], sin in [d/2:]
  const int* slots;      // [M] cache slot (-1: skip the K/V write)
  uint16_t* q_out;            // [M, nq, d]
  uint16_t* kc;               // [blocks, nkv, 16, d]
  uint16_t* vc;               // [blocks, nkv, d, 16]
  // non-null (decode): V rows go here row-major [M][v_ld] (16-B stores) instead of the V^T cache;
  // the decode attention kernel writes the newest token's V^T itself (attention.hip AttnArgs.v_new)
  uint16_t* v_rows;
  long v_ld;
  int nq, nkv, d;
  // PLAIN / RESADD / GELU: bias[n] added to the product before the epilogue op (null: none)
  const uint16_t* bias;
  // Grouped mode (MoE experts, csrc/kernels/moe.hip): a device tile list g_tiles
  // [expert | first row | rows] x g_max, then the live tile count at g_tiles[3 * g_max].  Row tile
  // i covers rows [first, first + rows) of Y (and of A, or A rows g_perm[r] / g_k: a gather), and
  // multiplies by W + expert * g_wstride.  M must be g_max * BM; splits 1.
  const int* g_tiles;
  int g_max;
  const int* g_perm;
  int g_k;
  long g_wstride;
  // 1: W is stored K-PANEL-MAJOR, [K / 64][N][64] (element (n, k) at ((k / 64) N + n) 64 + k % 64):
  // every ring fill of the weight operand (8 rows x 128 B) is then ONE contiguous 1 KB of the
  // weight stream instead of eight 128-B pieces 2K-11K bytes apart (HBM pages / L2 channels);
  // repacked once at load time (models/llama.py).  Not with the grouped (MoE) mode.
  int w_panel;
  // Stream-K decomposition (ops.gemm.stream_k_table): sk_grid workgroups, workgroup L (the
  // XCD-remapped block id) walks sk_table[L][0 .. sk_segmax) = int4 (tile, first k-step, end
  // k-step, slab index | contributors << 16), tile < 0 ends its list; split-K slabs hold sk_cmax
  // slots per tile.  Null: one (tile, split) unit per workgroup.
  const int* sk_table;
  int sk_grid, sk_segmax, sk_cmax;
  // k depth of a staged sub-tile: 0 / 64 (default), 32 (tgemm.hip by_tile_k32 plans)
  int kdepth;
  // MFMA of the wave tiles: 0 / 16 (mfma_f32_16x16x32_bf16, default), 32 (mfma_f32_32x32x16_bf16,
  // tgemm.hip by_tile_m32 plans)
  int mfma;
  // tile raster: 0 / 1 = n-major (consecutive workgroups of an XCD share a weight tile), G > 1 =
  // groups of G m-tile rows (an XCD's consecutive workgroups cover G m-tiles x (32 / G) n-tiles, so
  // they share G activation and 32 / G weight panels; tgemm.hip tgemm_kernel)
  int raster;
};
enum { EPI_PLAIN = 0, EPI_RESADD = 1, EPI_QKV = 2, EPI_SWIGLU = 3, EPI_GELU = 4 };
}  // namespace dllm
