"""Llama-family decoder (TinyLlama, Llama-3.x, Phi-3, Mixtral MoE) on the HIP op library.

One module covers every BASELINE.json family: they differ only in shapes, RoPE parameters,
tied embeddings and dense-vs-MoE MLP (models.configs).  MI355X-first layout decisions:
  * fused QKV weight [(nq + 2 nkv) d, H] and fused gate|up weight [2 I, H] — one GEMM each, on
    the LDS-tiled MFMA GEMM with fused epilogues (csrc/kernels/tgemm.hip; the fused-epilogue
    GEMV at batch <= 8; hipBLASLt core + a standalone epilogue only where the autotuner measured
    that faster, ops/gemm.py);
  * RMSNorm folded into the consuming GEMM and RoPE + the paged K / V^T write in the QKV GEMM's
    epilogue (fused decoder layer below; ``DLLM_FUSED=0`` keeps the unfused reference layer:
    norm + residual kernel, RoPE + KV-write kernel, SiLU·mul, used for CPU parity);
  * the LM head runs only on the last position of each sequence;
  * tensor parallel (Megatron column/row split): QKV / gate|up column-parallel, o_proj /
    down_proj row-parallel + ONE all-reduce each (or reduce-scatter + all-gather under sequence
    parallelism), vocab-parallel embedding (masked lookup + all-reduce) and LM head (distributed
    arg-max / top-k; parallel.comm).
Weights: random init with a fixed seed (no checkpoints in this environment) or HF safetensors.

Fused decoder layer (GPU, any tensor-parallel size; ``DLLM_FUSED=0`` disables): the residual stream
``r`` is updated in place by GEMM epilogues (csrc/kernels/tgemm.hip) and every RMSNorm is folded
into the GEMM that consumes it (gamma into the weight columns, rinv from the producer's partial
row sums of squares), so a dense layer is five launches: QKV+RoPE+KV-write, attention,
o_proj+residual, gate|up+SwiGLU, down+residual.  Under tensor parallelism the column-parallel QKV and
gate|up keep their fused epilogues on this rank's heads / intermediate shard, and each row-parallel
projection (o_proj, down) writes its partial sums, which ONE collective all-reduces with the
residual add and the next RMSNorm's row statistics fused in (ParallelContext.all_reduce_resadd:
the one-shot IPC kernel for decode-size messages): seven launches per layer, no standalone norm,
RoPE or SiLU kernels.  The fused weights are stored instead of the plain ones (same bytes);
``reference_layers()`` reconstructs the plain layout for reference checks.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch

from .. import ops
from ..parallel.comm import SINGLE, ParallelContext, shard_range
from .configs import ModelConfig


@dataclass
class AttnMeta:
    """Per-forward attention metadata (all int32 device tensors)."""
    slots: torch.Tensor        # [T] cache slot per new token (-1: skip)
    block_tables: torch.Tensor  # [S, max_blocks]
    qstart: torch.Tensor       # [S]
    qlen: torch.Tensor         # [S]
    ctx: torch.Tensor          # [S]
    tile_seq: torch.Tensor     # [num_tiles]
    tile_tok0: torch.Tensor    # [num_tiles]
    last_idx: torch.Tensor     # [S] int64 index of each sequence's last new token in the packed batch
    splits: int = 1
    workspace: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
    split_len: Optional[torch.Tensor] = None  # int32 device scalar: dynamic split-K (opt-in)
    xcd_remap: bool = False                    # prefill: XCD-contiguous attention block order
    items: Optional[torch.Tensor] = None       # decode: persistent attention work list (ops.decode_work_items)
    grid_items: int = 0                        # workgroups walking ``items``
    flash: bool = False                        # prefill: tile_seq/tile_tok0 are 128-row flash tiles
    max_ctx: int = 0                           # prefill: longest context (host-known; flash split-KV choice)
    all_last: bool = False                     # decode: every row is its sequence's last token (no gather)


def qk_dim_order(d: int) -> torch.Tensor:
    """Row order of one q/k head in the fused QKV weight: 32-row groups holding dims
    16g..16g+15 then d/2+16g..d/2+16g+15, so each RoPE pair (i, i + d/2) lands in two adjacent
    16-column MFMA fragments of the same lane (tgemm EPI_QKV)."""
    idx = []
    for g in range(d // 32):
        idx += list(range(16 * g, 16 * g + 16)) + list(range(d // 2 + 16 * g, d // 2 + 16 * g + 16))
    return torch.tensor(idx, dtype=torch.long)


def gate_up_order(I: int) -> torch.Tensor:
    """Row order of the fused gate|up weight: 32-row groups of 16 gate rows then the 16 matching
    up rows (tgemm EPI_SWIGLU pairs them in-register)."""
    o = torch.arange(2 * I)
    g, c = o // 32, o % 32
    return torch.where(c < 16, 16 * g + c, I + 16 * g + (c - 16))


def _qkv_rows(nq: int, nkv: int, d: int) -> torch.Tensor:
    p = qk_dim_order(d)
    rows = [h * d + p for h in range(nq + nkv)] + [torch.arange((nq + nkv) * d, (nq + 2 * nkv) * d)]
    return torch.cat(rows)


def fuse_qkv_weight(wqkv: torch.Tensor, ln: torch.Tensor, nq: int, nkv: int, d: int) -> torch.Tensor:
    idx = _qkv_rows(nq, nkv, d).to(wqkv.device)
    return (wqkv.index_select(0, idx).float() * ln.float()[None, :]).to(wqkv.dtype).contiguous()


def unfuse_qkv_weight(wf: torch.Tensor, ln: torch.Tensor, nq: int, nkv: int, d: int) -> torch.Tensor:
    idx = _qkv_rows(nq, nkv, d).to(wf.device)
    out = torch.empty_like(wf, dtype=torch.float32)
    out[idx] = wf.float() / ln.float()[None, :]
    return out.to(wf.dtype)


def fuse_gate_up_weight(wgu: torch.Tensor, ln: torch.Tensor) -> torch.Tensor:
    idx = gate_up_order(wgu.shape[0] // 2).to(wgu.device)
    return (wgu.index_select(0, idx).float() * ln.float()[None, :]).to(wgu.dtype).contiguous()


def unfuse_gate_up_weight(wf: torch.Tensor, ln: torch.Tensor) -> torch.Tensor:
    idx = gate_up_order(wf.shape[0] // 2).to(wf.device)
    out = torch.empty_like(wf, dtype=torch.float32)
    out[idx] = wf.float() / ln.float()[None, :]
    return out.to(wf.dtype)


class LlamaModel:
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, par: ParallelContext = SINGLE,
                 seed: int = 0, weights: Optional[str] = None, init_std: float = 0.02):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.par = par
        tp, r = par.tp_size, par.tp_rank
        if cfg.n_heads % tp or cfg.n_kv_heads % tp or cfg.intermediate % tp or cfg.vocab % tp:
            raise ValueError(f"{cfg.name}: heads/kv_heads/intermediate/vocab must divide tp={tp}")
        self.nq = cfg.n_heads // tp
        self.nkv = cfg.n_kv_heads // tp
        self.d = cfg.head_dim
        self.I = cfg.intermediate // tp
        self.vocab_shard = shard_range(cfg.vocab, r, tp)
        # MoE sharding: TP-within-expert (default; one all-reduce, graph-capturable) and, with
        # DLLM_MOE_PARALLEL=ep, ALSO expert parallel for prefill-size batches (E/tp whole experts per
        # rank, all-to-all dispatch/combine: parallel.expert_parallel).  EP's split sizes are a host
        # sync, so decode steps (graph-captured) keep the TP-within-expert shards: both layouts are
        # resident (Mixtral TP=8: +11.6 GB per GPU, cheap on a 288 GB part)
        self.moe_ep = bool(cfg.is_moe and tp > 1 and (par.moe_ep or os.environ.get("DLLM_MOE_PARALLEL") == "ep"))
        self.ep_min_tokens = int(os.environ.get("DLLM_EP_MIN_TOKENS", "128"))
        self.ep_calls = 0
        if self.moe_ep and cfg.n_experts % tp:
            raise ValueError(f"{cfg.name}: n_experts {cfg.n_experts} must divide ep={tp}")
        self.expert_shard = shard_range(cfg.n_experts, r, tp) if self.moe_ep else slice(0, cfg.n_experts)
        self.scale = 1.0 / math.sqrt(self.d)
        self.layers: List[Dict[str, torch.Tensor]] = []
        self._init_random(seed, init_std)
        if weights:
            self.load_safetensors(weights)
        self.cos_sin = ops.rope_cos_sin(cfg.max_position, self.d, cfg.rope_theta, self.device, cfg.rope_scaling)
        self.fused = self._fusable()
        if self.fused:
            self._fuse_weights()
        # MoE experts on the grouped LDS-tiled GEMM (csrc/kernels/moe.hip moe_ffn_tg): gate/up rows
        # of every expert interleaved in place for the SwiGLU epilogue
        self.moe_tg = bool(cfg.is_moe and self.device.type == "cuda" and ops.native_available()
                           and cfg.hidden % 64 == 0 and self.I % 64 == 0)
        if self.moe_tg:
            idx = gate_up_order(self.I).to(self.device)
            for L in self.layers:
                L["w13"] = L["w13"].index_select(1, idx).contiguous()

    # ------------------------------------------------------------------ fused layout
    def _fusable(self) -> bool:
        cfg = self.cfg
        if self.device.type != "cuda" or os.environ.get("DLLM_FUSED", "1") != "1":
            return False
        if not ops.native_available():
            return False
        return (self.d % 32 == 0 and cfg.hidden % 64 == 0 and (self.nq * self.d) % 64 == 0
                and (cfg.is_moe or (self.I % 64 == 0)))

    PANEL_NAMES = ("wqkv_f", "wo", "wgu_f", "wd")

    def _fuse_weights(self) -> None:
        for L in self.layers:
            L["wqkv_f"] = fuse_qkv_weight(L.pop("wqkv"), L["ln1"], self.nq, self.nkv, self.d)
            if "wgu" in L:
                L["wgu_f"] = fuse_gate_up_weight(L.pop("wgu"), L["ln2"])
        # K-panel-major copies of the fused decoder GEMM weights (ops.gemm.panel_weight): the tgemm
        # plans stream them; the row-major weights stay for the GEMV / skinny / hipBLASLt paths.  Kept
        # only while the copies fit in a quarter of the device memory still FREE (e.g. not
        # Llama-3-70B at TP=1: 141 GB of weights on a 288 GB part; co-located engines and processes
        # sharing the GPU each see what the others left), and never in the one-GPU multi-rank
        # rehearsal (N processes would each add a copy on one card)
        if not ops.gemm.W_PANEL or self.device.type != "cuda" or os.environ.get("DLLM_REHEARSE_ONE_GPU") == "1":
            return
        names = [n for n in self.PANEL_NAMES if n in self.layers[0] and self.layers[0][n].shape[1] % 64 == 0]
        extra = sum(L[n].numel() * L[n].element_size() for L in self.layers for n in names)
        free, _ = torch.cuda.mem_get_info(self.device)
        if extra > 0.25 * free:
            return
        for L in self.layers:
            for n in names:
                L[n + "_p"] = ops.gemm.panel_weight(L[n])

    def reference_layers(self) -> List[Dict[str, torch.Tensor]]:
        """Layer weights in the plain (unfused) layout, e.g. for a CPU reference forward."""
        if not self.fused and not getattr(self, "moe_tg", False):
            return self.layers
        out = []
        for L in self.layers:
            R = {k: v for k, v in L.items() if k not in ("wqkv_f", "wgu_f") and not k.endswith("_p")}
            if "wqkv_f" in L:
                R["wqkv"] = unfuse_qkv_weight(L["wqkv_f"], L["ln1"], self.nq, self.nkv, self.d)
            if "wgu_f" in L:
                R["wgu"] = unfuse_gate_up_weight(L["wgu_f"], L["ln2"])
            out.append(R)
        if self.moe_tg:
            idx = gate_up_order(self.I).to(self.device)
            for R, L in zip(out, self.layers):
                w = torch.empty_like(L["w13"])
                w[:, idx] = L["w13"]
                R["w13"] = w
        return out

    # ------------------------------------------------------------------ weights
    def _init_random(self, seed: int, std: float) -> None:
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev if dev.type == "cuda" else "cpu")
        # every TP rank draws the SAME full tensor stream and keeps its shard -> TP == TP1 numerics
        g.manual_seed(seed)

        def rnd(*shape):
            return (torch.randn(*shape, generator=g, device=dev, dtype=torch.float32) * std).to(dt)

        H, d, nq, nkv = cfg.hidden, cfg.head_dim, cfg.n_heads, cfg.n_kv_heads
        tp, r = self.par.tp_size, self.par.tp_rank
        qs, ks = shard_range(nq * d, r, tp), shard_range(nkv * d, r, tp)
        isl = shard_range(cfg.intermediate, r, tp)
        emb_full = rnd(cfg.vocab, H)
        self.embed = emb_full[self.vocab_shard].contiguous()
        self.lm_head = self.embed if cfg.tie_embeddings else rnd(cfg.vocab, H)[self.vocab_shard].contiguous()
        del emb_full
        ones = torch.ones(H, device=dev, dtype=dt)
        for _ in range(cfg.n_layers):
            wq, wk, wv = rnd(nq * d, H), rnd(nkv * d, H), rnd(nkv * d, H)
            wo = rnd(H, nq * d)
            L = {"ln1": ones.clone(), "ln2": ones.clone(),
                 "wqkv": torch.cat([wq[qs], wk[ks], wv[ks]], 0).contiguous(),
                 "wo": wo[:, qs].contiguous()}
            if cfg.is_moe:
                E = cfg.n_experts
                L["wgate"] = rnd(E, H)
                w13, w2, w13e, w2e = [], [], [], []
                esl = self.expert_shard
                for e in range(E):  # every rank draws every expert (same stream), keeps its part
                    gate, up, down = rnd(cfg.intermediate, H), rnd(cfg.intermediate, H), rnd(H, cfg.intermediate)
                    w13.append(torch.cat([gate[isl], up[isl]], 0))
                    w2.append(down[:, isl])
                    if self.moe_ep and esl.start <= e < esl.stop:   # this rank's whole experts (EP prefill)
                        w13e.append(torch.cat([gate, up], 0))
                        w2e.append(down)
                L["w13"] = torch.stack(w13).contiguous()   # [E, 2I/tp, H]
                L["w2"] = torch.stack(w2).contiguous()     # [E, H, I/tp]
                if self.moe_ep:
                    L["w13_ep"] = torch.stack(w13e).contiguous()   # [E/tp, 2I, H]
                    L["w2_ep"] = torch.stack(w2e).contiguous()     # [E/tp, H, I]
            else:
                gate, up, down = rnd(cfg.intermediate, H), rnd(cfg.intermediate, H), rnd(H, cfg.intermediate)
                L["wgu"] = torch.cat([gate[isl], up[isl]], 0).contiguous()
                L["wd"] = down[:, isl].contiguous()
            self.layers.append(L)
        self.final_norm = ones.clone()

    def load_safetensors(self, path: str) -> None:
        """Load HF-format weights (a file or a directory of shards); keeps this rank's shard."""
        from safetensors import safe_open
        files = [path] if os.path.isfile(path) else sorted(
            os.path.join(path, f) for f in os.listdir(path) if f.endswith(".safetensors"))
        tensors: Dict[str, torch.Tensor] = {}
        for f in files:
            with safe_open(f, framework="pt", device="cpu") as fh:
                for k in fh.keys():
                    tensors[k] = fh.get_tensor(k)
        cfg, tp, r = self.cfg, self.par.tp_size, self.par.tp_rank
        d, nq, nkv = cfg.head_dim, cfg.n_heads, cfg.n_kv_heads
        qs, ks = shard_range(nq * d, r, tp), shard_range(nkv * d, r, tp)
        isl = shard_range(cfg.intermediate, r, tp)
        put = lambda t: t.to(self.device, self.dtype).contiguous()
        self.embed = put(tensors["model.embed_tokens.weight"][self.vocab_shard])
        self.lm_head = self.embed if cfg.tie_embeddings else put(tensors["lm_head.weight"][self.vocab_shard])
        self.final_norm = put(tensors["model.norm.weight"])
        for i, L in enumerate(self.layers):
            p = f"model.layers.{i}."
            L["ln1"] = put(tensors[p + "input_layernorm.weight"])
            L["ln2"] = put(tensors[p + "post_attention_layernorm.weight"])
            if p + "self_attn.qkv_proj.weight" in tensors:  # phi-3 fused layout
                w = tensors[p + "self_attn.qkv_proj.weight"]
                wq, wk, wv = w[:nq * d], w[nq * d:(nq + nkv) * d], w[(nq + nkv) * d:]
            else:
                wq, wk, wv = (tensors[p + f"self_attn.{n}_proj.weight"] for n in "qkv")
            L["wqkv"] = put(torch.cat([wq[qs], wk[ks], wv[ks]], 0))
            L["wo"] = put(tensors[p + "self_attn.o_proj.weight"][:, qs])
            if cfg.is_moe:
                pm = p + "block_sparse_moe."
                L["wgate"] = put(tensors[pm + "gate.weight"])
                esl = self.expert_shard

                def experts(fsl, rng):
                    return (put(torch.stack([torch.cat([tensors[pm + f"experts.{e}.w1.weight"][fsl],
                                                        tensors[pm + f"experts.{e}.w3.weight"][fsl]], 0)
                                             for e in rng])),
                            put(torch.stack([tensors[pm + f"experts.{e}.w2.weight"][:, fsl] for e in rng])))
                L["w13"], L["w2"] = experts(isl, range(cfg.n_experts))
                if self.moe_ep:
                    L["w13_ep"], L["w2_ep"] = experts(slice(0, cfg.intermediate), range(esl.start, esl.stop))
            elif p + "mlp.gate_up_proj.weight" in tensors:
                w = tensors[p + "mlp.gate_up_proj.weight"]
                I = cfg.intermediate
                L["wgu"] = put(torch.cat([w[:I][isl], w[I:][isl]], 0))
                L["wd"] = put(tensors[p + "mlp.down_proj.weight"][:, isl])
            else:
                L["wgu"] = put(torch.cat([tensors[p + "mlp.gate_proj.weight"][isl],
                                          tensors[p + "mlp.up_proj.weight"][isl]], 0))
                L["wd"] = put(tensors[p + "mlp.down_proj.weight"][:, isl])

    def weight_bytes(self) -> int:
        n = self.embed.numel() + (0 if self.lm_head is self.embed else self.lm_head.numel()) + self.final_norm.numel()
        for L in self.layers:   # one copy of each matrix: the K-panel copies ("_p") duplicate bytes, not reads
            n += sum(t.numel() for k, t in L.items() if not k.endswith("_p"))
        return n * self.embed.element_size()

    # ------------------------------------------------------------------ forward
    def _embed(self, ids: torch.Tensor) -> torch.Tensor:
        # HIP row gather; under TP each rank gathers its vocab shard (zero rows elsewhere) and the
        # all-reduce assembles the embeddings
        h = ops.embedding(ids, self.embed, self.vocab_shard.start)
        return self.par.all_reduce(h) if self.par.tp_size > 1 else h

    def _mlp(self, L, x: torch.Tensor) -> torch.Tensor:
        if not self.cfg.is_moe:
            return ops.linear_swiglu(ops.linear(x, L["wgu"]), L["wd"])
        return self._moe(L, x)

    def _moe(self, L, x: torch.Tensor) -> torch.Tensor:
        """Top-k expert FFN: HIP router kernel (fp32 projection + softmax top-k, batch-invariant)
        -> ops.moe_ffn (device-side token permutation + grouped expert GEMMs, no host sync, so
        decode steps stay graph-captured).  Experts are TP-sharded along I; the caller all-reduces
        the partial sums."""
        ids, w = ops.moe_router(x, L["wgate"], self.cfg.experts_per_token)
        if self.moe_tg:
            return ops.moe_ffn_tg(x, ids, w, L["w13"], L["w2"])
        return ops.moe_ffn(x, ids, w, L["w13"], L["w2"])

    def use_ep(self, T: int) -> bool:
        """Expert-parallel MoE for this batch: EP mode, a prefill-size batch, not inside a graph
        capture (EP's all-to-all split sizes are a host sync)."""
        return (self.moe_ep and T >= self.ep_min_tokens
                and not (self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()))

    def _mlp_out(self, L, x: torch.Tensor) -> torch.Tensor:
        """Complete (replicated) MLP output: TP partial sums all-reduced, or the expert-parallel
        path (token slice per rank -> all-to-all dispatch/combine -> all-gather)."""
        if not self.use_ep(x.shape[0]):
            return self.par.all_reduce(self._mlp(L, x))
        from ..parallel.expert_parallel import all_gather_rows, ep_moe_ffn, token_slice
        par, T = self.par, x.shape[0]
        lo, hi = token_slice(T, par.tp_rank, par.tp_size)
        xl = x[lo:hi]
        ids, w = ops.moe_router(xl, L["wgate"], self.cfg.experts_per_token)
        yl = ep_moe_ffn(xl, ids, w, L["w13_ep"], L["w2_ep"], self.cfg.n_experts, par.tp_group, par.tp_size)
        self.ep_calls += 1
        return all_gather_rows(yl, T, par.tp_group, par.tp_size)

    def _attention(self, q: torch.Tensor, kc: torch.Tensor, vc: torch.Tensor, meta: AttnMeta,
                   v_new: Optional[torch.Tensor] = None) -> torch.Tensor:
        if meta.flash:   # prefill: 128-row tiles, K/V staged once per workgroup (flash_prefill.hip)
            return ops.flash_attention(q, kc, vc, meta.block_tables, meta.qstart, meta.qlen, meta.ctx,
                                       meta.tile_seq, meta.tile_tok0, scale=self.scale, causal=True,
                                       max_ctx=meta.max_ctx)
        return ops.paged_attention(q, kc, vc, meta.block_tables, meta.qstart, meta.qlen, meta.ctx,
                                   meta.tile_seq, meta.tile_tok0, scale=self.scale, causal=True,
                                   splits=meta.splits, workspace=meta.workspace, split_len=meta.split_len,
                                   xcd_remap=meta.xcd_remap, items=meta.items, grid_items=meta.grid_items,
                                   v_new=v_new)

    def hidden_states(self, input_ids: torch.Tensor, positions: torch.Tensor, meta: AttnMeta,
                      kv_caches: List[Tuple[torch.Tensor, torch.Tensor]],
                      scatter: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
        """Final-normed hidden states of each sequence's last new token: [S, H].  ``scatter`` =
        (block tables, update pairs): a decode step's block-table updates, applied before any
        attention reads the tables (by the fused path's embedding launch itself)."""
        cfg = self.cfg
        if getattr(self, "fused", False):
            return self._hidden_states_fused(input_ids, positions, meta, kv_caches, scatter=scatter)
        if scatter is not None:
            ops.scatter_pairs(*scatter)
        if self.par.use_sp(input_ids.shape[0]) and not (input_ids.is_cuda and torch.cuda.is_current_stream_capturing()):
            return self._hidden_states_sp(input_ids, positions, meta, kv_caches)
        h = self._embed(input_ids)
        residual = torch.zeros_like(h)
        spare = torch.empty_like(h)   # ping-pong partner: a fused norm+GEMV writes the new residual here
        for li, L in enumerate(self.layers):
            qkv, res = ops.norm_linear(h, residual, spare, L["ln1"], cfg.rms_eps, L["wqkv"])
            residual, spare = res, (spare if res is residual else residual)
            kc, vc = kv_caches[li]
            q = ops.rope_and_cache(qkv, positions, self.cos_sin, meta.slots, kc, vc, self.nq, self.nkv, self.d)
            o = self._attention(q, kc, vc, meta)
            h = self.par.all_reduce(ops.linear(o.view(o.shape[0], -1), L["wo"]))
            if not self.cfg.is_moe:
                gu, res = ops.norm_linear(h, residual, spare, L["ln2"], cfg.rms_eps, L["wgu"])
                residual, spare = res, (spare if res is residual else residual)
                h = self.par.all_reduce(ops.linear_swiglu(gu, L["wd"]))
            else:
                x = ops.rms_norm(h, L["ln2"], cfg.rms_eps, residual=residual)
                h = self._mlp_out(L, x)
        last_h = h if meta.all_last else h.index_select(0, meta.last_idx)
        last_r = residual if meta.all_last else residual.index_select(0, meta.last_idx)
        return ops.rms_norm(last_h, self.final_norm, cfg.rms_eps, residual=last_r)

    def _hidden_states_fused(self, input_ids: torch.Tensor, positions: torch.Tensor, meta: AttnMeta,
                             kv_caches: List[Tuple[torch.Tensor, torch.Tensor]],
                             scatter: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
        """Fused layer path (module docstring): residual stream ``r`` updated in place by GEMM
        epilogues; ``ssq``/``n`` = partial row sums of r^2 of the latest residual producer."""
        cfg, par = self.cfg, self.par
        T, H, eps = input_ids.shape[0], cfg.hidden, cfg.rms_eps
        slots_n = max(ops.gemm.max_slots(H, T), 32)   # >= the one-shot all-reduce's column slices
        ssq_a = torch.empty((slots_n, T), dtype=torch.float32, device=input_ids.device)
        ssq_b = torch.empty((slots_n, T), dtype=torch.float32, device=input_ids.device)
        tp = par.tp_size > 1
        # sequence parallelism (DLLM_SEQ_PARALLEL=1, prefill-size batches, eager only): every
        # row-parallel reduction becomes reduce-scatter + residual add on the token slice +
        # all-gather (ParallelContext.sp_resadd)
        sp = tp and par.use_sp(T) and not (input_ids.is_cuda and torch.cuda.is_current_stream_capturing())
        resadd = par.sp_resadd if sp else par.all_reduce_resadd
        if not tp:
            # the gather also leaves each row's sum of squares in slot 0 (first layer's row scale)
            r = ops.embedding(input_ids, self.embed, self.vocab_shard.start, ssq_out=ssq_a[0], scatter=scatter)
            n = 1
        else:
            # vocab-parallel rows (zero outside this rank's shard) summed by the all-reduce, which
            # also leaves the row statistics of the first RMSNorm
            r = torch.empty((T, H), dtype=self.dtype, device=input_ids.device)
            n = par.all_reduce_resadd(ops.embedding(input_ids, self.embed, self.vocab_shard.start, scatter=scatter),
                                      r, ssq_a, add=False)
        # decode (one new token per sequence, TP 1, head_dim 64): the QKV GEMM hands V over row-major
        # and the attention kernel writes each sequence's newest V^T itself (ops.gemm.qkv_rope_cache;
        # for d = 96 / 128 the patch would cost the attention kernel a wave per SIMD)
        vn = (torch.empty((T, self.nkv * self.d), dtype=self.dtype, device=input_ids.device)
              if (not tp and self.d == 64 and meta.all_last and meta.items is not None and input_ids.is_cuda)
              else None)
        for li, L in enumerate(self.layers):
            kc, vc = kv_caches[li]
            # column-parallel QKV (this rank's heads) with RMSNorm folded + RoPE + paged K/V write
            q = ops.gemm.qkv_rope_cache(r, L["wqkv_f"], ssq_a, n, eps, positions, self.cos_sin, meta.slots, kc, vc,
                                        self.nq, self.nkv, self.d, wp=L.get("wqkv_f_p"), v_new=vn)
            v_new = None
            if vn is not None:
                q, v_new = q
            o = self._attention(q, kc, vc, meta, v_new=v_new)
            if not tp:
                nb = ops.gemm.matmul_resadd(o.view(T, -1), L["wo"], r, ssq_b, wp=L.get("wo_p"))
            else:   # row-parallel o_proj: partial sums -> all-reduce + residual add + row statistics
                nb = resadd(ops.linear(o.view(T, -1), L["wo"], wp=L.get("wo_p")), r, ssq_b)
            if not cfg.is_moe:
                act = ops.gemm.swiglu_matmul(r, L["wgu_f"], ssq_b, nb, eps, wp=L.get("wgu_f_p"))
                if not tp:
                    n = ops.gemm.matmul_resadd(act, L["wd"], r, ssq_a, wp=L.get("wd_p"))
                else:
                    n = resadd(ops.linear(act, L["wd"], wp=L.get("wd_p")), r, ssq_a)
            else:
                x = ops.rms_norm(r, L["ln2"], eps)
                if not tp:
                    n = ops.gemm.res_add_ssq(self._mlp(L, x), r, ssq_a)
                elif self.use_ep(T):   # expert parallel: the combined output is already replicated
                    n = ops.gemm.res_add_ssq(self._mlp_out(L, x), r, ssq_a)
                else:               # TP-within-expert partial sums
                    n = resadd(self._mlp(L, x), r, ssq_a)
        return ops.rms_norm(r if meta.all_last else r.index_select(0, meta.last_idx), self.final_norm, eps)

    def _hidden_states_sp(self, input_ids: torch.Tensor, positions: torch.Tensor, meta: AttnMeta,
                          kv_caches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        """Sequence-parallel TP forward (Megatron-SP) for prefill-size batches.

        The residual stream and both RMSNorms of every layer live on this rank's 1/tp token slice;
        each row-parallel output (wo, down / MoE) is reduce-scattered to the slice instead of
        all-reduced, and the normed slice is all-gathered before the column-parallel projection
        (wqkv, gate|up). Same bytes on the wire as the all-reduces it replaces, but the norm work
        and the [T, H] residual/activation buffers shrink by tp (long prompts: SURVEY §5.7)."""
        cfg, par = self.cfg, self.par
        T = input_ids.shape[0]
        from ..parallel.expert_parallel import token_slice
        lo, hi = token_slice(T, par.tp_rank, par.tp_size)
        # embedding shards are vocab-parallel partial sums: reduce-scatter them straight to the slice
        h = par.reduce_scatter_rows(ops.embedding(input_ids, self.embed, self.vocab_shard.start))
        residual = torch.zeros_like(h)
        for li, L in enumerate(self.layers):
            x = par.all_gather_rows(ops.rms_norm(h, L["ln1"], cfg.rms_eps, residual=residual), T)
            qkv = ops.linear(x, L["wqkv"])
            kc, vc = kv_caches[li]
            q = ops.rope_and_cache(qkv, positions, self.cos_sin, meta.slots, kc, vc, self.nq, self.nkv, self.d)
            o = self._attention(q, kc, vc, meta)
            h = par.reduce_scatter_rows(ops.linear(o.view(o.shape[0], -1), L["wo"]))
            x = par.all_gather_rows(ops.rms_norm(h, L["ln2"], cfg.rms_eps, residual=residual), T)
            if self.use_ep(T):
                h = self._mlp_out(L, x)[lo:hi]
            else:
                h = par.reduce_scatter_rows(self._mlp(L, x))
        h = par.all_gather_rows(h, T)
        residual = par.all_gather_rows(residual, T)
        last_h = h.index_select(0, meta.last_idx)
        last_r = residual.index_select(0, meta.last_idx)
        return ops.rms_norm(last_h, self.final_norm, cfg.rms_eps, residual=last_r)

    def logits(self, hidden: torch.Tensor) -> torch.Tensor:
        """This rank's vocab shard of the logits: [S, V / tp] (bf16)."""
        return ops.linear(hidden, self.lm_head)

    def greedy(self, hidden: torch.Tensor) -> torch.Tensor:
        """Distributed arg-max over the vocab-parallel LM head -> token ids [S] int32."""
        lg = self.logits(hidden)
        if self.par.tp_size == 1:
            return ops.argmax(lg)
        loc = ops.argmax(lg)
        val = lg.gather(1, loc.long().unsqueeze(1)).float().squeeze(1)
        pair = torch.stack([val, (loc + self.vocab_shard.start).float()], dim=1)  # ids < 2^24: exact in f32
        allp = self.par.all_gather(pair)                    # [tp, S, 2]
        best = allp[..., 0].argmax(dim=0)                   # first max -> lowest rank -> lowest id
        return allp[..., 1].gather(0, best.unsqueeze(0)).squeeze(0).to(torch.int32)

    def sample(self, hidden: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, top_k: torch.Tensor,
               seed: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """Fused per-row sampling (greedy / exact top-k + top-p, ops.sample_rows) over the LM head.

        Under TP the vocab is sharded: every rank reduces its shard to its ranked top-256
        (value, global id) pairs (ops.tp_candidates, one launch), one all-gather of [tp, S, 256, 2]
        replaces the [S, V] logits, and every rank merges the tp sorted lists and draws with the
        same seed (ops.tp_sample, one launch) -> the same token on all ranks, and the token the
        unsharded sampler would draw (the global top-k of any k <= 256 is inside the union of the
        per-shard top-256).  Graph-capturable: three launches, no host sync, no torch.topk."""
        lg = self.logits(hidden)
        if self.par.tp_size == 1:
            return ops.sample_rows(lg, temperature, top_p, top_k, seed, out=out)
        cand = ops.tp_candidates(lg, self.vocab_shard.start)
        return ops.tp_sample(self.par.all_gather(cand), temperature, top_p, top_k, seed, out=out)

    def topk_candidates(self, hidden: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Global top-k (values desc, ids) from per-rank top-k of the vocab shards."""
        lg = self.logits(hidden).float()
        k_loc = min(k, lg.shape[1])
        v, i = torch.topk(lg, k_loc, dim=-1)
        i = i + self.vocab_shard.start
        if self.par.tp_size > 1:
            av, ai = self.par.all_gather(v), self.par.all_gather(i)   # [tp, S, k]
            v = av.permute(1, 0, 2).reshape(v.shape[0], -1)
            i = ai.permute(1, 0, 2).reshape(i.shape[0], -1)
            v, j = torch.topk(v, min(k, v.shape[1]), dim=-1)
            i = i.gather(1, j)
        return v.contiguous(), i.contiguous()
