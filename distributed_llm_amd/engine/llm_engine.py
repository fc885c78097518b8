"""LLM serving engine: paged KV cache, prefix caching, continuous batching, hipGraph decode.

Replaces the reference's external Ollama/llama.cpp engine (the hot loop of
§3.2).  Structure:
  * ``BlockManager`` (native, csrc/runtime/block_manager.cpp) — 16-token KV blocks with
    hash-chained prefix caching: a new turn of a conversation reuses the previous turn's KV;
  * scheduler — FIFO admission, chunked prefill under a token budget, prefill-first, then
    one decode step for every running sequence (continuous batching);
  * decode runner — each running sequence owns a ROW of persistent per-row metadata
    (block table row, context length) on the device; a decode step uploads ONE small packed
    int32 buffer and replays a hipGraph captured for the batch-size bucket (model forward +
    LM head + the fused per-row sampler: arg-max or top-k/top-p, ops.sample_rows), so the host
    cost per step is O(batch) numpy work + one memcpy + one graph launch + one token read-back;
  * prefill runner — eager (shapes vary), packed variable-length batch, attention over the
    cached prefix + new tokens with the same paged kernel.
KV memory is sized for 288 GB HBM3E parts: ``kv_cache_gb`` (default: 60 % of free memory).
"""
from __future__ import annotations

import itertools
import math
import os
import threading
import time
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from .. import ops
from ..models.configs import ModelConfig, get_model_config
from ..models.llama import AttnMeta, LlamaModel
from ..utils.faults import diag, fault
from ..parallel.comm import SINGLE, ParallelContext
from ..utils.tracing import tracer
from .sampling import SamplingParams
from .tokenizer import get_tokenizer

try:
    from . import _runtime  # type: ignore
except ImportError as _e:  # pragma: no cover - build step missing
    _runtime = None
    _runtime_err = _e

BS = ops.BLOCK_SIZE


def _need_runtime():
    if _runtime is None:
        raise RuntimeError(f"native runtime not built ({_runtime_err}); run `python -m distributed_llm_amd._build`")
    return _runtime


@dataclass
class RequestOutput:
    request_id: int
    text: str
    token_ids: List[int]
    num_prompt: int
    num_cached: int
    num_generated: int
    latency_ms: float
    ttft_ms: float
    queue_ms: float
    decode_tok_s: float
    error: Optional[str] = None

    @property
    def num_prefill(self) -> int:
        return self.num_prompt - self.num_cached


KV_RESERVE_GB = 16.0   # device memory left free next to a requested KV pool (_alloc_kv)


@dataclass
class _Seq:
    id: int
    prompt: List[int]
    params: SamplingParams
    arrival: float
    out: List[int] = field(default_factory=list)
    fill: List[int] = field(default_factory=list)   # tokens to (re)compute on admission: prompt + out
    num_cached: int = 0
    num_computed: int = 0
    row: int = -1
    text: Optional[str] = None
    admitted: Optional[float] = None
    first_tok: Optional[float] = None
    finished: Optional[float] = None
    error: Optional[str] = None
    done: threading.Event = field(default_factory=threading.Event)
    out_text: Optional[str] = None   # detokenised answer, formed as soon as the sequence stops
    released: bool = False           # blocks and row returned (_release)
    notify: Optional[Callable[["_Seq"], None]] = None   # called with the sequence once it is done

    def finish(self) -> None:
        """Mark done: wakes ``done`` waiters, then hands the sequence to ``notify`` (an event-driven
        client's completion queue), so one client thread never has to poll hundreds of handles.
        Idempotent: a row that stops inside a pipelined burst is finished early (``_complete_early``)
        and again when its blocks are released; ``notify`` fires only on the first call."""
        if self.done.is_set():
            return
        self.done.set()
        if self.notify is not None:
            self.notify(self)

    @property
    def length(self) -> int:
        return len(self.prompt) + len(self.out)


def decode_buckets(R: int, mode: Optional[str] = None) -> List[int]:
    """Batch sizes that get a captured decode graph (a step runs the smallest bucket >= its batch).

    Powers of two up to 64, then every 32 rows to 256, then every 64 rows (``fine``, default).
    A decode batch drains continuously as conversations finish, so with power-of-two buckets a
    step at 300 rows ran the 512-row graph: the weight GEMMs above 128 rows scale with M and paid
    for up to 40 % padding.  ``pow2`` (DLLM_BUCKETS=pow2) restores the coarse ladder.
    """
    mode = mode or os.environ.get("DLLM_BUCKETS", "fine")
    if mode == "pow2":
        ladder = [1 << i for i in range(0, 20)]
    else:
        ladder = [1, 2, 4, 8, 16, 32, 48, 64] + list(range(96, 257, 32)) + list(range(320, 1 << 16, 64))
    return [b for b in ladder if b < R] + [R]


class LLMEngine:
    def __init__(self, model: Union[str, ModelConfig], device: str = "cuda", par: ParallelContext = SINGLE,
                 kv_cache_gb: Optional[float] = None, max_num_seqs: int = 256, max_model_len: Optional[int] = None,
                 max_prefill_tokens: int = 16384, prefix_cache: bool = True, use_graphs: bool = True,
                 seed: int = 0, weights: Optional[str] = None, tokenizer: Optional[str] = None):
        self.cfg = get_model_config(model) if isinstance(model, str) else model
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None and torch.cuda.is_available():
            # an explicit index: worker threads call torch.cuda.set_device(self.device), which
            # rejects a bare "cuda" (the background loop died on it before serving anything)
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.par = par
        self.model = LlamaModel(self.cfg, device=self.device, par=par, seed=seed, weights=weights)
        self.tok = get_tokenizer(self.cfg.vocab, self.cfg.bos_id, self.cfg.eos_id, tokenizer)
        self.max_model_len = min(max_model_len or self.cfg.max_position, self.cfg.max_position)
        self.max_num_seqs = max_num_seqs
        self.max_prefill_tokens = max_prefill_tokens
        self.max_blocks = (self.max_model_len + BS - 1) // BS
        self._alloc_kv(kv_cache_gb)
        self.bm = _need_runtime().BlockManager(self.num_blocks, BS, prefix_cache, int(self.KV_PLACEMENT))
        self._ids = itertools.count()
        self._lock = threading.Lock()          # held by the thread currently driving the step loop
        self._inbox: List[_Seq] = []            # submitted, not yet seen by the driver
        self._inbox_lock = threading.Lock()
        self._inbox_cv = threading.Condition(self._inbox_lock)
        # Set from the moment a pipelined burst decides to end until the next decode step is on
        # the GPU: the step loop's host work (drain, release, admission, staging) is then all that
        # stands between the GPU and its next work, so an in-process client thread (the bench's
        # routing driver) can hold off its own Python work meanwhile instead of contending for the
        # GIL (profiles/r4_driver_window_gaps.md).
        self.host_critical = threading.Event()
        self._driving = False
        self._bg: Optional[threading.Thread] = None   # background step-loop thread (start())
        self._bg_stop = False
        self._active: List[_Seq] = []
        self._mirror = None                     # TP lockstep channel (enable_tp_mirror)
        self._mirror_pending = None
        self._memo: "OrderedDict[str, List[int]]" = OrderedDict()
        self._memo_cap = 200_000
        self._memo_lock = threading.Lock()
        self.on_gpu = self.device.type == "cuda"
        self._ws_owner = ("engine", id(self))   # split-K workspaces of this engine's kernels/graphs
        # expert-parallel MoE exchanges split sizes on the host (parallel.expert_parallel): eager
        # (an expert-parallel MoE model decodes on its TP-within-expert shards: graph-capturable)
        self.use_graphs = use_graphs and self.on_gpu
        self._gen = torch.Generator(device=self.device if self.on_gpu else "cpu")
        self._gen.manual_seed(seed + 1)
        self._seed_base = (seed * 0x9E3779B1 + 0x5851F42D) & 0x7FFFFFFF
        self._init_rows()
        if self.on_gpu and os.environ.get("DLLM_AUTOTUNE", "1") == "1":
            self._autotune()      # DLLM_AUTOTUNE=0: heuristic GEMM plans (multi-process tests on one GPU)
        self._graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self._graph_pool = None
        self.collective_trips = 0
        self.trip_steps: List[int] = []   # decode-step counter at each collective trip
        self._check_graph_collectives()
        self.steps = {"prefill": 0, "decode": 0, "prefill_tokens": 0, "decode_tokens": 0}
        self.timers = {"prefill": 0.0, "decode_host_pre": 0.0, "decode_gpu_wait": 0.0, "decode_host_post": 0.0,
                       "encode": 0.0, "admit": 0.0, "output": 0.0, "complete": 0.0}
        # step-loop timers (disjoint): prefill, admit, decode_host_pre / gpu_wait / host_post, complete
        # (answers detokenised under the next step); caller-side: encode (submit), output (results)

    # ------------------------------------------------------------------ setup
    def _alloc_kv(self, kv_cache_gb: Optional[float]) -> None:
        m, L = self.model, self.cfg.n_layers
        per_block = L * 2 * m.nkv * BS * m.d * 2
        if kv_cache_gb is None:
            if self.device.type == "cuda":
                free, _ = torch.cuda.mem_get_info(self.device)
                kv_cache_gb = 0.6 * free / 2**30
            else:
                kv_cache_gb = 0.25
        elif self.device.type == "cuda":
            # a requested size is an upper bound: what is free after this engine's weights (and any
            # engine or TP shard already on the device), less KV_RESERVE_GB for graphs, split-K
            # workspaces, prefill activations and the router encoder (a 160 GB default
            # pool next to Llama-3-70B TP shards must not over-commit the 288 GB part)
            free, _ = torch.cuda.mem_get_info(self.device)
            kv_cache_gb = min(float(kv_cache_gb), max(0.5, free / 2**30 - KV_RESERVE_GB))
        self.kv_cache_gb = float(kv_cache_gb)
        self.num_blocks = max(int(kv_cache_gb * 2**30) // per_block, self.max_blocks + 8)
        self.k_cache = torch.empty((L, self.num_blocks, m.nkv, BS, m.d), dtype=m.dtype, device=self.device)
        self.v_cache = torch.empty((L, self.num_blocks, m.nkv, m.d, BS), dtype=m.dtype, device=self.device)
        self.kv_caches = [(self.k_cache[i], self.v_cache[i]) for i in range(L)]

    def _init_rows(self) -> None:
        R = self.max_num_seqs
        self.R = R
        self._free_rows = list(range(R - 1, -1, -1))
        self._pf_host = self._pf_dev = self._pf_evt = None   # prefill input staging (_stage_i32)
        self._h2d_ring = None                                 # small pinned copies (_small_h2d)
        self._h2d_i = 0
        self._early_pf = None      # a prefill chunk queued under the last step of a decode burst
        self._pf_tok: Optional[torch.Tensor] = None   # pinned first tokens of a prefill chunk
        self._in_join_burst = False
        # DLLM_DIAG=sync: per pipelined step (host prep s, wait for the in-flight step s, launched)
        self._sync_log: Optional[list] = [] if diag("sync") else None
        pin = self.on_gpu
        # host mirror of the device block table (pinned); row R is the dummy row of padding tiles.
        self.bt_host_t = torch.zeros((R + 1, self.max_blocks), dtype=torch.int32, pin_memory=pin)
        self.bt_host = self.bt_host_t.numpy()
        self.bt_dev = torch.zeros((R + 1, self.max_blocks), dtype=torch.int32, device=self.device)
        self._bt_dirty = True          # whole-table copy needed (admissions / releases)
        self._bt_hw = 0                # block-table columns ever used (the host -> device copy width)
        self._bt_rows = [R + 1, -1]    # [lo, hi] rows rewritten since the last sync (async copy range)
        self._bt_upd: List[int] = []   # (flat index, block) pairs applied inside the decode graph
        self.buckets = decode_buckets(R)
        mb = self.buckets[-1]
        # packed decode buffer: ids | pos | slots | tile_seq  (mb each) | qstart | qlen | ctx (R+1 each)
        #                       | attention split length
        #                       | sampler: temperature, top_p (f32 bits), top_k (mb each) | seed
        #                       | id sources (mb: row of the previous step's d_out, -1 = ids above)
        #                       | block-table updates [n, (flat idx, block) * R]
        s0 = 4 * mb + 3 * (R + 1) + 1
        o = [0, mb, 2 * mb, 3 * mb, 4 * mb, 4 * mb + R + 1, 4 * mb + 2 * (R + 1), 4 * mb + 3 * (R + 1),
             s0 + 4 * mb + 1, s0 + 3 * mb + 1]
        self._dec_n = o[8] + 1 + 2 * R
        # Step I/O by kernels inside the step's graph (ops.step_fetch / step_store: the pinned
        # buffers are device-mapped), not by async copies: an H2D copy runs on an SDMA engine and
        # waited ~320 us per step for the previous step's read-back to signal it (r4 gap analysis).
        self._gio = self.on_gpu and ops.native_available()   # step I/O by kernels inside the step graph
        self.dec_dev = torch.zeros(self._dec_n, dtype=torch.int32, device=self.device)
        # two pinned staging buffers: the pipelined decode (_decode_burst) fills one while the
        # previous step's async copy may still be reading the other
        self._dec_bufs = []
        for _ in range(2):
            t = torch.zeros(self._dec_n, dtype=torch.int32, pin_memory=pin)
            t[o[9]:o[9] + mb] = -1
            self._dec_bufs.append((t, t.numpy(), t.numpy().view(np.float32)))
        self.dec_host_t, self.dec_host, self.dec_host_f = self._dec_bufs[0]
        self._off = o
        self._so = s0
        # the whole sampler runs inside the decode graph (ops.sample_rows) unless the vocab is
        # tensor-parallel (then the distributed arg-max / top-k of LlamaModel is used)
        # one-launch sampler inside the decode graph (TP: merged per-shard top-256 candidates, LlamaModel.sample)
        self.fused_sampler = True   # one-launch in-graph sampler (the host-side path stays for tests)
        self._seed_ctr = 0
        dv = self.dec_dev
        self.d_temp = dv[s0:s0 + mb].view(torch.float32)
        self.d_topp = dv[s0 + mb:s0 + 2 * mb].view(torch.float32)
        self.d_topk = dv[s0 + 2 * mb:s0 + 3 * mb]
        self.d_seed = dv[s0 + 3 * mb:s0 + 3 * mb + 1]
        self.d_split = self.dec_dev[o[7]:o[7] + 1]
        self.d_upd = self.dec_dev[o[8]:]
        d = self.dec_dev
        self.d_ids, self.d_pos, self.d_slots, self.d_tseq = (d[o[0]:o[1]], d[o[1]:o[2]], d[o[2]:o[3]], d[o[3]:o[4]])
        self.d_qstart, self.d_qlen, self.d_ctx = d[o[4]:o[5]], d[o[5]:o[6]], d[o[6]:o[6] + R + 1]
        self.d_tok0 = torch.zeros(mb, dtype=torch.int32, device=self.device)
        self.d_last = torch.arange(mb, dtype=torch.int64, device=self.device)
        # sampled tokens; slot [bucket] of a TP decode step holds the collectives' health vote
        self.d_out = torch.zeros(mb + 1, dtype=torch.int32, device=self.device)
        self.d_src = torch.zeros(mb, dtype=torch.int64, device=self.device)   # pipelined: id gather rows
        self._out_bufs = [torch.zeros(mb + 1, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        # numpy views of the pinned read-back buffers: ndarray.tolist() of a step's tokens costs a few
        # us, torch's Tensor.tolist() ~0.4 ms (it was the largest host item of a pipelined step)
        self._out_np = [b.numpy() for b in self._out_bufs]
        self._src_bufs = [torch.zeros(mb, dtype=torch.int64, pin_memory=pin) for _ in range(2)]
        self._out_evts = [torch.cuda.Event() for _ in range(2)] if self.on_gpu else None
        self.d_hidden = torch.zeros((mb, self.cfg.hidden), dtype=self.model.dtype, device=self.device)
        nkv, dh = self.model.nkv, self.model.d
        self.max_splits = 16
        ws = mb * nkv * self.max_splits * 16
        self.dec_ws = (torch.empty(ws * dh, dtype=torch.float32, device=self.device),
                       torch.empty(ws * 2, dtype=torch.float32, device=self.device),
                       torch.zeros(mb * nkv + 2, dtype=torch.int32, device=self.device))
        # persistent decode attention: host-built work list, copied with the step's metadata
        self.attn_worklist = self.ATTN_WORKLIST and not self.ATTN_DYNAMIC
        if self.attn_worklist:
            cap = 4 + 4 * mb * nkv * self.max_splits   # extended list (ops.decode_work_items)
            self._items_bufs = []
            for _ in range(2):
                t = torch.zeros(cap, dtype=torch.int32, pin_memory=pin)
                self._items_bufs.append((t, t.numpy()))
            self.items_host_t, self.items_host = self._items_bufs[0]
            self.items_dev = torch.zeros(cap, dtype=torch.int32, device=self.device)

    def _autotune(self) -> None:
        """Pick the fastest GEMM plan for every decode bucket and weight shape (before capture)."""
        m = self.model
        shapes = set()
        L = m.layers[0]
        for name in ("wqkv", "wqkv_f", "wo", "wgu", "wgu_f"):
            if name in L:
                shapes.add((L[name].shape[0], L[name].shape[1], False))
        if "wd" in L:
            # fused layers stream the SwiGLU activation as a plain operand (EPI_RESADD)
            shapes.add((L["wd"].shape[0], L["wd"].shape[1], not m.fused))
        shapes.add((m.lm_head.shape[0], m.lm_head.shape[1], False))
        fused = [tuple(L[n].shape) for n in ("wqkv_f", "wo", "wgu_f", "wd") if m.fused and n in L]
        with ops.gemm.workspace_owner(self._ws_owner):
            ops.gemm_autotune(sorted(shapes), [b for b in self.buckets if b <= ops.gemm.MAX_M], self.device,
                              verbose=os.environ.get("DLLM_VERBOSE") == "1", fused=fused,
                              qkv_dims=(m.nq, m.nkv, m.d) if fused else None,
                              qkv_cache=self.kv_caches[0] if fused else None)
            ops.gemm.reserve(self.device)

    # Decode attention split-K.  Default: a static split count sized to the batch (_splits_for),
    # tiles ordered longest context first (the dispatcher then starts the longest chains first).
    # ATTN_DYNAMIC (class attribute, off): fixed grid depth, and each step the host writes a split
    # length so the batch yields ~ATTN_TARGET_WGS workgroups; measured slower on MI355X because
    # surplus early-exit blocks cost dispatch slots (csrc/kernels/attention.hip note).
    ATTN_DYNAMIC = False
    SORT_TILES = True        # decode tiles longest context first
    ATTN_TARGET_WGS = 2048
    # Default: persistent work-list attention (ops.decode_work_items): a fixed grid of at most
    # ATTN_PGRID workgroups walks ~ATTN_ITEMS_PER_WG equal key ranges each, longest first.
    ATTN_WORKLIST = True
    ATTN_PGRID = 512
    ATTN_ITEMS_PER_WG = 1
    # Work list at every batch size: in a whole decode step (scripts/microbench.py decode, 1x
    # MI355X, TinyLlama) it cut B=1 from 1.14 to 0.89 ms and B=16 from 1.51 to 1.29 ms vs the
    # static split grid (a kernel-only sweep had B=16-64 about even)
    ATTN_WL_MIN_BS = 1
    # shortest key range of one work-list unit (split-K granularity)
    # (256: with the parallel split combine, batch 1-8 steps at 2k context are 2-3 % faster than at
    # 512 and equal at 8k, microbench decode sweep; it only matters while batch x context < 64k
    # tokens, above that the target unit count sets the chunk)
    ATTN_MIN_CHUNK = 256
    def _use_worklist(self, bs: int) -> bool:
        return self.attn_worklist and bs >= self.ATTN_WL_MIN_BS

    def _attn_grid(self, bs: int) -> int:
        return int(max(1, min(self.ATTN_PGRID, bs * self.model.nkv * self.max_splits)))

    def _decode_splits(self, bs: int) -> int:
        if self.ATTN_DYNAMIC:
            return 8 if bs <= 64 else 4
        return self._splits_for(bs)

    def _split_len(self, total_ctx: int) -> int:
        per = total_ctx * self.model.nkv / max(1, self.ATTN_TARGET_WGS)
        return int(max(256, math.ceil(per / 256) * 256))

    def _splits_for(self, tiles: int) -> int:
        # measured on MI355X (scripts/microbench.py attn): split-K pays only while tiles x kv-heads
        # leaves CUs idle; at >= 256 work units one split is fastest.
        return int(max(1, min(8, math.ceil(256 / max(1, tiles * self.model.nkv)))))

    # ------------------------------------------------------------------ public API
    def encode(self, text: str) -> List[int]:
        """Tokenise a prompt, re-using the exact token ids of the longest previously served
        prompt+response text that prefixes it (session memo).

        A chat turn's prompt is the previous turn's prompt + the model's reply + the new user
        message.  Re-tokenising the reply text does not, in general, give back the token ids the
        model generated (and whose KV blocks are cached); re-using the generated ids makes the
        whole previous turn a prefix-cache hit, so only the new user message is prefilled.
        """
        memo = self._memo
        if memo:
            pos = len(text)
            for _ in range(64):  # message boundaries, newest first
                pos = text.rfind("\n", 0, pos)
                if pos <= 0:
                    break
                with self._memo_lock:
                    ids = memo.get(text[:pos])
                    if ids is not None:
                        memo.move_to_end(text[:pos])
                if ids is not None:
                    return list(ids) + self.tok.encode(text[pos:], add_bos=False)
        return self.tok.encode(text)

    def _remember(self, text: str, ids: List[int]) -> None:
        with self._memo_lock:
            self._memo[text] = ids
            while len(self._memo) > self._memo_cap:
                self._memo.popitem(last=False)

    def generate(self, prompts: Sequence[Union[str, List[int]]],
                 params: Union[SamplingParams, Sequence[SamplingParams], None] = None) -> List[RequestOutput]:
        """Run a batch of requests to completion with continuous batching."""
        seqs = self._make_seqs(prompts, params)
        self._submit_and_wait([s for s in seqs if s.error is None])
        return self.results(seqs)

    def submit(self, prompts: Sequence[Union[str, List[int]]],
               params: Union[SamplingParams, Sequence[SamplingParams], None] = None,
               notify: Optional[Callable[["_Seq"], None]] = None) -> List["_Seq"]:
        """Enqueue requests WITHOUT waiting (the background loop, ``start()``, must be running):
        returns handles whose ``done`` event is set when each request has finished; ``results``
        turns them into outputs.  An event-driven client (bench.py turn pipelining) keeps the
        continuous batch full from one thread this way instead of one blocked thread per request.
        ``notify(seq)`` is called (from the engine's loop thread) when a submitted request finishes;
        requests rejected here (``error`` already set) are returned done and are not notified."""
        if self._bg is None:
            raise RuntimeError("submit() needs the background loop (start())")
        seqs = self._make_seqs(prompts, params)
        live = [s for s in seqs if s.error is None]
        for s in live:
            s.notify = notify
        with self._inbox_lock:
            self._inbox.extend(live)
            self._inbox_cv.notify()
        return seqs

    def results(self, seqs: Sequence["_Seq"]) -> List[RequestOutput]:
        _t = time.perf_counter()
        outs = [self._output(s) for s in seqs]
        self.timers["output"] += time.perf_counter() - _t
        return outs

    def _make_seqs(self, prompts: Sequence[Union[str, List[int]]],
                   params: Union[SamplingParams, Sequence[SamplingParams], None]) -> List["_Seq"]:
        if params is None:
            params = SamplingParams()
        plist = list(params) if isinstance(params, (list, tuple)) else [params] * len(prompts)
        now = _t = time.perf_counter()
        seqs: List[_Seq] = []
        for p, sp in zip(prompts, plist):
            ids = self.encode(p) if isinstance(p, str) else list(p)
            s = _Seq(next(self._ids), ids, sp, now)
            s.text = p if isinstance(p, str) else None
            limit = self.max_model_len - max(1, sp.max_new_tokens)
            if len(ids) > limit:  # keep the most recent context (left truncation)
                s.prompt = ids[:1] + ids[len(ids) - limit + 1:]
            if len(s.prompt) == 0 or limit <= 1:
                s.error = "prompt too long for max_model_len"
                s.finish()
            seqs.append(s)
        self.timers["encode"] += time.perf_counter() - _t
        return seqs

    def _submit_and_wait(self, seqs: List[_Seq]) -> None:
        """Continuous batching across callers (leader/follower): requests from concurrent threads
        (HTTP handlers, pool dispatchers) join ONE running batch.  The first caller to find the
        engine idle drives the step loop until every submitted sequence is done; later callers
        only enqueue and wait — their sequences are admitted at the driver's next step."""
        if self.par.enabled and self._mirror is None:
            # TP ranks without a mirror channel: every rank calls generate() with the same
            # requests in the same order (lockstep by construction, no cross-caller merging)
            with self._lock:
                self._run(seqs)
            return
        with self._inbox_lock:
            self._inbox.extend(seqs)
            lead = not self._driving    # always False while a background loop owns the driver role
            if lead:
                self._driving = True
            self._inbox_cv.notify()
        if lead:
            with self._lock:
                try:
                    self._run([])
                except BaseException as e:
                    self._abort_all(f"engine step failed: {e!r}")
                    raise
        for s in seqs:
            s.done.wait()

    def _abort_all(self, why: str) -> None:
        """A failed step must not strand followers: fail every admitted/queued sequence."""
        with self._inbox_lock:
            pending, self._inbox = self._inbox, []
            self._driving = self._bg is not None
        for s in pending + list(self._active):
            # early-completed rows (_complete_early) are done but still own blocks and a row
            if not s.done.is_set() or s.row >= 0:
                if not s.done.is_set():
                    s.error = s.error or why
                try:
                    self.bm.free(s.id)
                except Exception:  # noqa: BLE001 - best effort cleanup
                    pass
                if s.row >= 0:
                    self.bt_host[s.row].fill(0)
                    self._free_rows.append(s.row)
                    s.row = -1
                s.finish()
        self._active = []
        self._early_pf = None
        self.host_critical.clear()
        self._bt_dirty = True

    # TP mirror: admissions are exchanged every MIRROR_EVERY scheduler iterations (and whenever the
    # batch is empty), not every decode step: leader and members call _take_inbox at the same points
    # of the same deterministic schedule, so both sides know when a broadcast comes
    MIRROR_EVERY = max(1, int(os.environ.get("DLLM_TP_ADMIT_EVERY", "8")))

    def _take_inbox(self, final: bool) -> List[_Seq]:
        if self._mirror is not None:
            self._mirror_iter += 1
            poll = final or self._mirror_iter >= self._mirror_due
            if not poll:
                return []
            self._mirror_due = self._mirror_iter + self.MIRROR_EVERY
            if not self._mirror[2]:
                return self._mirror_take()
        with self._inbox_lock:
            new, self._inbox = self._inbox, []
            if final and not new and self._bg is None:
                self._driving = False   # atomically with the empty check: no submission is lost
        if self._mirror is not None:    # TP leader: members replay exactly this admission
            self._mirror_send({"seqs": [[s.id, s.prompt, s.params.to_dict()] for s in new]})
        return new

    # ------------------------------------------------------------------ tensor-parallel lockstep
    def enable_tp_mirror(self, group, leader: int) -> "LLMEngine":
        """Continuous batching for a tensor-parallel pool.

        Every TP rank must run identical scheduler decisions (same admissions, same batch, same
        collectives).  The leader (the rank that receives requests) broadcasts, every
        ``MIRROR_EVERY`` scheduler iterations (and whenever the batch is empty), the requests it
        takes from its inbox — sequence id, prompt token ids, sampling parameters — over
        ``group`` (a CPU/gloo group of the TP ranks); members replay them in ``follow()``.  Scheduling is deterministic given those inputs (block manager, stop rules,
        seeded sampling), so the members' engines stay in step while concurrent callers keep
        joining the leader's running batch (instead of one lockstep batch at a time)."""
        import torch.distributed as dist
        self._mirror = (group, leader, dist.get_rank() == leader)
        self._mirror_iter = 0
        self._mirror_due = self.MIRROR_EVERY   # next poll (iterations; a pipelined burst counts its steps)
        return self

    def _mirror_send(self, msg) -> None:
        from ..parallel import p2p
        p2p.bcast_obj(msg, self._mirror[1], self._mirror[0])

    def _mirror_recv(self):
        from ..parallel import p2p
        return p2p.bcast_obj(None, self._mirror[1], self._mirror[0])

    def _mirror_take(self) -> List[_Seq]:
        msg, self._mirror_pending = self._mirror_pending, None
        if msg is None:
            msg = self._mirror_recv()
        if "seqs" not in msg:
            raise RuntimeError(f"TP mirror out of step: expected an admission, got {msg!r}")
        now = time.perf_counter()
        return [_Seq(int(i), list(p), SamplingParams.from_dict(sp), now) for i, p, sp in msg["seqs"]]

    def mirror_control(self, msg) -> None:
        """Leader: a control message (``{"sync": True}`` / ``{"stop": True}``) for the members,
        sent between scheduler runs (holds the step lock)."""
        if self._mirror is None or not self._mirror[2]:
            return
        with self._lock:
            self._mirror_send(msg)

    def follow(self, on_sync=None) -> None:
        """Member: replay the leader's scheduler until it sends stop."""
        if self._mirror is None or self._mirror[2]:
            raise RuntimeError("follow() is for TP members with a mirror channel")
        if self.on_gpu:
            torch.cuda.set_device(self.device)
        while True:
            msg = self._mirror_recv()
            if msg.get("stop"):
                return
            if msg.get("sync"):
                if on_sync is not None:
                    on_sync()
                continue
            self._mirror_pending = msg
            with self._lock:
                try:
                    self._run([])
                except BaseException as e:  # noqa: BLE001 - same recovery as the leader's loop
                    # the leader catches the same step failure (every rank raises it on the same
                    # step, e.g. a custom all-reduce trip) and aborts its batch; a member that
                    # exited here would leave the leader's next collective waiting forever
                    self._abort_all(f"engine step failed: {e!r}")

    # ------------------------------------------------------------------ background serving loop
    def start(self) -> "LLMEngine":
        """Serve from a dedicated step-loop thread (server mode).

        Leader/follower driving (``_submit_and_wait``) makes the first caller run the loop until
        the engine drains, so under a continuous stream of requests that caller's own request is
        held back until every other caller is done.  With a background loop callers only enqueue
        and wait for THEIR sequences: a conversation can submit its next turn while the rest of
        the batch is still decoding (turn pipelining, bench.py --pipeline)."""
        if self.par.enabled and (self._mirror is None or not self._mirror[2]):
            return self   # TP members follow the leader's scheduler (follow())
        with self._inbox_lock:
            if self._bg is not None:
                return self
            if self._driving:
                raise RuntimeError("start() while a caller is driving the step loop")
            self._bg_stop = False
            self._driving = True          # the loop thread owns the driver role from now on
            self._bg = threading.Thread(target=self._bg_loop, name=f"dllm-engine-{self.cfg.name}",
                                        daemon=True)
            self._bg.start()
        return self

    def stop(self, timeout: float = 60.0) -> None:
        """Finish queued work, then end the background loop (callers drive again afterwards)."""
        with self._inbox_lock:
            t = self._bg
            if t is None:
                return
            self._bg_stop = True
            self._inbox_cv.notify_all()
        t.join(timeout)
        with self._inbox_lock:
            self._bg = None
            self._driving = False
        if self._mirror is not None and self._mirror[2]:
            self.mirror_control({"stop": True})

    def _bg_loop(self) -> None:
        if self.on_gpu:
            torch.cuda.set_device(self.device)
        while True:
            with self._inbox_lock:
                while not self._inbox and not self._bg_stop:
                    self._inbox_cv.wait()
                if not self._inbox and self._bg_stop:
                    return
            with self._lock:
                try:
                    self._run([])
                except BaseException as e:  # fail the affected requests, keep serving
                    self._abort_all(f"engine step failed: {e!r}")

    def stats(self) -> Dict[str, object]:
        st = dict(self.bm.stats())
        st.update(self.steps)
        st.update({f"t_{k}_s": round(v, 4) for k, v in self.timers.items()})
        st["model"] = self.cfg.name
        st["kv_blocks"] = self.num_blocks
        return st

    # ------------------------------------------------------------------ scheduling
    def _run(self, seqs: List[_Seq]) -> None:
        waiting = [s for s in seqs if s.error is None]
        prefilling: List[_Seq] = []
        running: List[_Seq] = []
        while True:
            waiting.extend(self._take_inbox(final=not (waiting or prefilling or running)))
            self._active = waiting + prefilling + running
            if not (waiting or prefilling or running):
                self.host_critical.clear()
                break
            # admit
            self._admit(waiting, prefilling, len(running))
            if not (prefilling or running):
                if waiting:  # nothing fits even alone -> fail the head request
                    s = waiting.pop(0)
                    s.error = "insufficient KV cache for request"
                    s.finish()
                continue
            if prefilling:
                _t = time.perf_counter()
                with tracer.span("engine.prefill", "engine", seqs=len(prefilling)):
                    if self._early_pf is not None:   # launched under the last step of a burst
                        h, self._early_pf = self._early_pf, None
                        done = self._prefill_finish(h)
                    else:
                        done = self._prefill_step(prefilling)
                self.timers["prefill"] += time.perf_counter() - _t
                for s in done:
                    prefilling.remove(s)
                    if self._finished(s):
                        self._release(s)
                    elif s.error == "__preempt__":
                        # no block for its first generated token: re-queue before it reaches a
                        # decode step (its slot would otherwise point at an unowned block)
                        self._release(s, keep=False)
                        s.error = None
                        waiting.insert(0, s)
                    else:
                        running.append(s)
                continue
            with tracer.span("engine.decode", "engine", batch=len(running)):
                if self._pipeline_ok():
                    finished, preempted = self._decode_burst(running, waiting, prefilling)
                else:
                    finished, preempted = self._decode_step(running)
            if tracer.enabled:
                tracer.counter("engine.batch", running=len(running), waiting=len(waiting),
                               free_kv_blocks=self.bm.num_free_blocks())
            if finished or preempted:
                _t = time.perf_counter()
                gone = set(map(id, finished)) | set(map(id, preempted))
                running[:] = [s for s in running if id(s) not in gone]
                for s in finished:
                    self._release(s)
                # out of KV blocks for a running sequence: preempt it and re-queue it
                for s in preempted:
                    self._release(s, keep=False)
                    s.error = None
                    waiting.insert(0, s)  # re-admitted with fill = prompt + out (recompute)
                self.timers["decode_host_post"] += time.perf_counter() - _t

    def _admit(self, waiting: List[_Seq], prefilling: List[_Seq], n_running: int, reserve_blocks: int = 0) -> None:
        """Move waiting requests that fit (a free row, KV blocks for prompt + 1) to ``prefilling``.
        ``reserve_blocks``: free blocks held back for running rows that are about to open a new block
        (an admission under a running burst must not take the block a continuing row reserves next)."""
        _ta = time.perf_counter()
        margin = reserve_blocks * BS
        while waiting and self._free_rows and len(prefilling) + n_running < self.R:
            s = waiting[0]
            s.fill = s.prompt + s.out
            if not self.bm.can_allocate(len(s.fill) + 1 + margin):
                break
            table, cached = self.bm.allocate(s.id, s.fill)
            if not table:
                break
            waiting.pop(0)
            s.num_cached = s.num_computed = cached
            s.admitted = time.perf_counter()
            s.row = self._free_rows.pop()
            self._set_row_blocks(s)
            prefilling.append(s)
        self.timers["admit"] += time.perf_counter() - _ta

    def _finished(self, s: _Seq) -> bool:
        if s.error is not None and s.error != "__preempt__":
            return True
        if not s.out:
            return False
        if len(s.out) >= s.params.max_new_tokens:
            return True
        if not s.params.ignore_eos and s.out[-1] == self.tok.eos_id:
            return True
        return s.length >= self.max_model_len

    def _release(self, s: _Seq, keep: bool = True) -> None:
        if s.released:              # already released inside a decode burst (BURST_JOIN)
            return
        s.released = keep
        if keep:
            if s.finished is None:    # _complete_early may have set it when the row stopped
                s.finished = time.perf_counter()
            if tracer.enabled:
                self._trace_request(s)
        self.bm.free(s.id)
        if keep:
            s.finish()
        if s.row >= 0:
            self.bt_host[s.row].fill(0)
            self._mark_bt_row(s.row)
            self._free_rows.append(s.row)
            s.row = -1

    def _trace_request(self, s: _Seq) -> None:
        lane = f"req {s.id % 64:02d}"   # 64 rotating lanes keep concurrent requests readable
        args = dict(id=s.id, prompt=len(s.prompt), cached=s.num_cached, generated=len(s.out))
        adm = s.admitted or s.finished
        tracer.complete("request.queue", s.arrival, adm, lane=lane, **args)
        if s.first_tok:
            tracer.complete("request.prefill", adm, s.first_tok, lane=lane, **args)
            tracer.complete("request.decode", s.first_tok, s.finished, lane=lane, **args)

    def _set_row_blocks(self, s: _Seq) -> None:
        t = self.bm.block_table(s.id)
        self.bt_host[s.row, :len(t)] = t
        self._bt_hw = max(self._bt_hw, len(t))
        self._bt_dirty = True
        self._mark_bt_row(s.row)

    def _mark_bt_row(self, row: int) -> None:
        lo, hi = self._bt_rows
        self._bt_rows = [min(lo, row), max(hi, row)]

    def _note_upd_cols(self) -> None:
        """Widen the host -> device block-table copy to every column a queued update writes."""
        if self._bt_upd:
            cols = np.asarray(self._bt_upd[0::2], dtype=np.int64) % self.max_blocks
            self._bt_hw = max(self._bt_hw, int(cols.max()) + 1)

    def _sync_bt(self, non_blocking: bool = False) -> None:
        """Host block table -> device (the columns any row has used) when admissions / releases
        changed it.  ``non_blocking`` (inside a decode burst that admits, BURST_JOIN): an async
        copy from the pinned mirror, stream-ordered before the next step; the host may rewrite a
        row before the copy runs only by admitting into it (which queues another copy) or by
        opening a new block (which the step's in-graph scatter applies as well)."""
        if self._bt_dirty and non_blocking:
            # whole rows of the pinned mirror are contiguous, so this copy really is asynchronous
            # (a column slice would be staged through pageable memory, which waits for the stream:
            # ADVICE r4); the range spans every row rewritten since the last sync, and queued
            # per-step updates of other rows are applied by the step's own in-graph scatter
            lo, hi = self._bt_rows
            if hi >= lo:
                self.bt_dev[lo:hi + 1].copy_(self.bt_host_t[lo:hi + 1], non_blocking=True)
            self._bt_rows = [self.bt_host_t.shape[0], -1]
            self._bt_dirty = False   # (_bt_upd stays queued for the next step's scatter)
            return
        if self._bt_dirty:
            # rare (admission / release): synchronous copy of the columns any row has used (a 128K
            # context table is 8K columns; a 2K-token batch needs 128 of them), which also subsumes
            # the queued per-step updates
            self._note_upd_cols()
            hw = min(self._bt_hw, self.max_blocks)
            if hw == self.max_blocks:
                self.bt_dev.copy_(self.bt_host_t, non_blocking=False)
            elif hw > 0:
                self.bt_dev[:, :hw].copy_(self.bt_host_t[:, :hw], non_blocking=False)
            self._bt_rows = [self.bt_host_t.shape[0], -1]
            self._bt_dirty = False
            self._bt_upd.clear()

    # ------------------------------------------------------------------ sampling
    def _next_seed(self) -> int:
        self._seed_ctr += 1
        return (self._seed_ctr * 0x2545F491 + self._seed_base) & 0x7FFFFFFF

    def _fill_sampler(self, h: np.ndarray, hf: np.ndarray, base: int, stride: int, seqs: List[_Seq], pad: int) -> None:
        """Per-row sampler parameters into a packed int32 buffer: temperature | top_p | top_k
        (``stride`` apart) and the step seed; rows [len(seqs), pad) are greedy padding."""
        n = len(seqs)
        ps = [s.params for s in seqs]
        hf[base:base + n] = np.fromiter((p.temperature for p in ps), dtype=np.float32, count=n)
        hf[base + stride:base + stride + n] = np.fromiter((p.top_p for p in ps), dtype=np.float32, count=n)
        h[base + 2 * stride:base + 2 * stride + n] = np.fromiter((p.top_k for p in ps), dtype=np.int32, count=n)
        if pad > n:
            hf[base + n:base + pad] = 0.0
        h[base + 3 * stride] = self._next_seed()

    def _sample(self, hidden: torch.Tensor, seqs: List[_Seq], greedy_ids: Optional[torch.Tensor],
                launch_only: bool = False) -> Union[List[int], torch.Tensor]:
        """Token per row.  ``launch_only`` (fused sampler): return the device tensor of tokens
        without waiting for it (the caller reads it back later)."""
        n = len(seqs)
        dev = hidden.device
        if self.fused_sampler:   # one launch: arg-max / top-k / top-p per row
            buf = np.zeros(3 * n + 1, dtype=np.int32)
            self._fill_sampler(buf, buf.view(np.float32), 0, n, seqs, n)
            t = self._small_h2d(buf) if self.on_gpu else torch.from_numpy(buf).to(dev)
            out = torch.empty(n, dtype=torch.int32, device=dev)
            out = self.model.sample(hidden[:n], t[:n].view(torch.float32), t[n:2 * n].view(torch.float32),
                                    t[2 * n:3 * n], t[3 * n:], out)
            return out if launch_only else out.tolist()
        ids = greedy_ids[:n] if greedy_ids is not None else self.model.greedy(hidden[:n])
        sampled = [i for i, s in enumerate(seqs) if not s.params.greedy]
        if not sampled:
            return ids.tolist()
        # only the sampled rows go through top-k + nucleus sampling; greedy rows keep the arg-max
        sel = torch.tensor(sampled, dtype=torch.int64, device=dev)
        k = max(seqs[i].params.k for i in sampled)
        vals, idx = self.model.topk_candidates(hidden.index_select(0, sel), k)
        prm = torch.tensor([[seqs[i].params.temperature, seqs[i].params.top_p, float(seqs[i].params.k)]
                            for i in sampled], dtype=torch.float32).to(dev, non_blocking=True)
        if any(seqs[i].params.k < vals.shape[1] for i in sampled):  # per-row top-k cut
            cols = torch.arange(vals.shape[1], device=dev, dtype=torch.float32)[None, :]
            vals = torch.where(cols < prm[:, 2:3], vals, torch.full_like(vals, -float("inf")))
        u = torch.rand(len(sampled), generator=self._gen, device=dev)
        if self.par.tp_size > 1:  # every TP rank must draw the same token
            self.par.all_reduce(u)
            u /= self.par.tp_size
        picks = ops.sample_top_p(vals, idx, prm[:, 0].contiguous(), prm[:, 1].contiguous(), u)
        out = ids.clone()
        out.index_copy_(0, sel, picks.to(out.dtype))
        return out.tolist()

    # ------------------------------------------------------------------ prefill
    def _prefill_step(self, prefilling: List[_Seq]) -> List[_Seq]:
        return self._prefill_finish(self._prefill_launch(prefilling))

    def _prefill_launch(self, prefilling: List[_Seq]) -> tuple:
        """Queue one prefill chunk (and the fused first-token sampler) on the GPU; the host does
        not wait.  ``_prefill_finish`` reads the first tokens back."""
        with ops.gemm.workspace_owner(self._ws_owner):
            return self._prefill_step_inner(prefilling)

    def _prefill_finish(self, handle: tuple) -> List[_Seq]:
        done_seqs, toks = handle
        if isinstance(toks, tuple):       # (pinned tokens, event): wait for the chunk only
            buf, ev = toks
            ev.synchronize()
            toks = buf.numpy()[:len(done_seqs)].tolist()
        elif torch.is_tensor(toks):
            toks = toks.tolist()          # the fused sampler's device output: waits for the chunk
        now = time.perf_counter()
        for s, tok in zip(done_seqs, toks):
            if s.first_tok is None:
                s.first_tok = now
            self._append(s, tok)
        return done_seqs

    def _prefill_step_inner(self, prefilling: List[_Seq]) -> tuple:
        budget = self.max_prefill_tokens
        chunk: List[tuple] = []
        for s in prefilling:
            if budget <= 0:
                break
            n = min(len(s.fill) - s.num_computed, budget)
            chunk.append((s, s.num_computed, s.num_computed + n))
            budget -= n
        ids, pos, slots, qstart, qlen, ctx, last = [], [], [], [], [], [], []
        G = self.model.nq // self.model.nkv
        flash = self.on_gpu and ops.flash_supported(self.model.d, G, self.max_blocks)
        tiler = ops.flash_tiles if flash else ops.build_tiles
        tseq, ttok = [], []
        t = 0
        for i, (s, a, b) in enumerate(chunk):
            ids.extend(s.fill[a:b])
            pos.extend(range(a, b))
            slots.extend(self.bm.slots(s.id, a, b))
            qstart.append(t)
            qlen.append(b - a)
            ctx.append(b)
            t += b - a
            last.append(t - 1)
            ts, tt = tiler([b - a], G)
            tseq.extend([i] * len(ts))
            ttok.extend(tt)
        nb = max((ctx_i + BS - 1) // BS for ctx_i in ctx)
        rows = np.fromiter((s.row for s, _, _ in chunk), dtype=np.int64, count=len(chunk))
        bt = self.bt_host[rows, :nb]
        dev = self.device
        splits = self._splits_for(len(tseq))
        if self.on_gpu:
            # one pinned staging buffer, one async H2D copy: the host builds this chunk while the
            # GPU still runs the previous one (per-tensor torch.tensor(..., device) copies sync)
            (slots_d, qstart_d, qlen_d, ctx_d, tseq_d, ttok_d, last_d, ids_d, pos_d, bt_d) = self._stage_i32(
                [slots, qstart, qlen, ctx, tseq, ttok, last, ids, pos, bt])
            last_d = last_d.to(torch.int64)
            bt_d = bt_d.view(len(chunk), nb)
        else:
            T = lambda x, dt=torch.int32: torch.tensor(x, dtype=dt, device=dev)
            slots_d, qstart_d, qlen_d, ctx_d, tseq_d, ttok_d = T(slots), T(qstart), T(qlen), T(ctx), T(tseq), T(ttok)
            last_d, ids_d, pos_d, bt_d = T(last, torch.int64), T(ids), T(pos), torch.from_numpy(np.ascontiguousarray(bt))
        meta = AttnMeta(slots=slots_d, block_tables=bt_d, qstart=qstart_d, qlen=qlen_d,
                        ctx=ctx_d, tile_seq=tseq_d, tile_tok0=ttok_d, last_idx=last_d,
                        splits=splits, xcd_remap=True, flash=flash, max_ctx=max(ctx))
        hidden = self.model.hidden_states(ids_d, pos_d, meta, self.kv_caches)
        if not self._collectives_ok():
            # a one-shot all-reduce timed out on some rank: every rank re-runs the chunk on RCCL
            # (same inputs, the K/V slot writes are idempotent)
            hidden = self.model.hidden_states(ids_d, pos_d, meta, self.kv_caches)
        self.steps["prefill"] += 1
        self.steps["prefill_tokens"] += t
        done_seqs = [s for (s, a, b) in chunk if b == len(s.fill)]
        for s, a, b in chunk:
            s.num_computed = b
            self.bm.commit(s.id, b)
        if not done_seqs:
            return [], []
        sel = [i for i, (s, a, b) in enumerate(chunk) if b == len(s.fill)]
        if len(sel) == len(chunk):
            h = hidden
        else:
            sel_a = np.asarray(sel, dtype=np.int32)
            sel_d = self._small_h2d(sel_a) if self.on_gpu else torch.from_numpy(sel_a)
            h = hidden.index_select(0, sel_d.to(torch.int64))
        toks = self._sample(h, done_seqs, None, launch_only=True)
        if self.on_gpu and torch.is_tensor(toks):
            # first tokens to pinned memory + an event: the host reads them once the chunk is done
            # without synchronising the stream (decode steps may be queued behind the chunk)
            n = len(done_seqs)
            if self._pf_tok is None or self._pf_tok.numel() < n:
                self._pf_tok = torch.empty(max(n, self.R), dtype=torch.int32, pin_memory=True)
            self._pf_tok[:n].copy_(toks[:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            return done_seqs, (self._pf_tok, ev)
        return done_seqs, toks

    def _small_h2d(self, a: np.ndarray) -> torch.Tensor:
        """A few KB of int32 to the device without a host stall: through a ring of 4 pinned slots
        (a slot is rewritten only after the copy that last read it has completed, which is long
        past by then), never through pageable memory (a pageable async copy may wait for the
        stream, i.e. for the decode step a prefill is queued behind)."""
        n = a.size
        if self._h2d_ring is None or self._h2d_ring[0][0].numel() < n:
            cap = max(1 << 14, 1 << (int(n) - 1).bit_length())
            self._h2d_ring = [(torch.empty(cap, dtype=torch.int32, pin_memory=True),
                               torch.empty(cap, dtype=torch.int32, device=self.device), None) for _ in range(4)]
            self._h2d_i = 0
        i = self._h2d_i
        self._h2d_i = (i + 1) % len(self._h2d_ring)
        host, dev, ev = self._h2d_ring[i]
        if ev is not None:
            ev.synchronize()
        host.numpy()[:n] = a.reshape(-1)
        dev[:n].copy_(host[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._h2d_ring[i] = (host, dev, ev)
        return dev[:n]

    def _stage_i32(self, parts) -> List[torch.Tensor]:
        """Pack int sequences / arrays into one pinned int32 buffer and copy it to the device with
        ONE non-blocking copy; returns device views in ``parts`` order.  The previous copy's event
        guards the pinned buffer against being rewritten while its DMA is still reading it."""
        arrs = [np.asarray(p, dtype=np.int32).ravel() for p in parts]
        total = sum(a.size for a in arrs)
        if self._pf_host is None or self._pf_host.numel() < total:
            if self._pf_evt is not None:
                self._pf_evt.synchronize()
            cap = max(1 << 16, 1 << (int(total) - 1).bit_length())
            self._pf_host = torch.empty(cap, dtype=torch.int32, pin_memory=True)
            self._pf_dev = torch.empty(cap, dtype=torch.int32, device=self.device)
        elif self._pf_evt is not None:
            self._pf_evt.synchronize()
        hn = self._pf_host.numpy()
        off, bounds = 0, []
        for a in arrs:
            hn[off:off + a.size] = a
            bounds.append((off, a.size))
            off += a.size
        self._pf_dev[:total].copy_(self._pf_host[:total], non_blocking=True)
        self._pf_evt = torch.cuda.Event()
        self._pf_evt.record()
        return [self._pf_dev[o:o + n] for o, n in bounds]

    def _append(self, s: _Seq, tok: int) -> None:
        s.out.append(int(tok))
        if self._finished(s):
            return
        slot = self.bm.append_token(s.id, int(tok))
        if slot < 0:
            s.error = "__preempt__"
            return
        nblk = (s.length + BS - 1) // BS
        blk = slot // BS
        if self.bt_host[s.row, nblk - 1] != blk:
            self.bt_host[s.row, nblk - 1] = blk
            self._bt_upd.extend((s.row * self.max_blocks + nblk - 1, blk))

    # ------------------------------------------------------------------ decode
    def _bucket(self, n: int) -> int:
        for b in self.buckets:
            if b >= n:
                return b
        raise ValueError(f"batch {n} exceeds max_num_seqs")

    def _prep_decode(self, running: List[_Seq], lens: np.ndarray, last: Optional[np.ndarray], p: int,
                     src: Optional[List[int]] = None) -> int:
        """Stage one decode step's inputs in pinned buffer ``p`` (the step's graph fetches them, or,
        without step I/O kernels, an async copy moves them).

        ``lens``: context length per row including the input token (position = lens - 1);
        ``last``: the input token per row, or None when it is the previous step's sampled token
        still on the device (pipelined decode): then ``src[i]`` is the row of ``d_out`` holding
        row i's input token.  Returns the step's bucket."""
        B = len(running)
        bs = self._bucket(B)
        o = self._off
        _, h, hf = self._dec_bufs[p]
        R = self.R
        rows = np.fromiter((s.row for s in running), dtype=np.int64, count=B)
        pos = lens - 1
        blocks = self.bt_host[rows, pos // BS].astype(np.int64)
        h[o[0]:o[0] + bs] = 0
        if last is not None:
            h[o[0]:o[0] + B] = last
        h[o[1]:o[1] + bs] = 0
        h[o[1]:o[1] + B] = pos
        h[o[2]:o[2] + bs] = -1
        h[o[2]:o[2] + B] = blocks * BS + pos % BS
        h[o[3]:o[3] + bs] = R            # padding tiles -> dummy row (qlen 0)
        order = np.argsort(-lens, kind="stable") if (self.SORT_TILES or self._use_worklist(bs)) else None
        h[o[3]:o[3] + B] = rows[order] if order is not None else rows
        n_items = 0
        if self._use_worklist(bs):
            grid = self._attn_grid(bs)
            target = self.ATTN_ITEMS_PER_WG * grid
            items_t, items = self._items_bufs[p]
            ops.decode_work_items(lens[order], self.model.nkv, self.max_splits, target,
                                  min_chunk=self.ATTN_MIN_CHUNK, out=items, seq=rows[order], qstart=order)
            n_items = ops.work_items_len(items)
        h[o[4]:o[6] + R + 1] = 0
        h[o[4] + rows] = np.arange(B)
        h[o[5] + rows] = 1
        h[o[6] + rows] = lens
        self._sync_bt(non_blocking=self._in_join_burst)
        h[o[7]] = self._split_len(int(lens.sum()))
        if self.fused_sampler:
            self._fill_sampler(h, hf, self._so, self.buckets[-1], running, bs)
        nu = len(self._bt_upd) // 2
        h[o[8]] = nu
        if nu:
            h[o[8] + 1:o[8] + 1 + 2 * nu] = self._bt_upd
            # the graph writes these columns on the device: count them in the copy width, or a
            # released row's stale device columns past it would survive the next admission sync
            self._note_upd_cols()
            self._bt_upd.clear()
        h[o[9]:o[9] + bs] = -1
        if src is not None:
            h[o[9]:o[9] + B] = src
        if self._gio:
            return bs               # the step's first kernel (ops.step_fetch) reads buffer p
        self.dec_dev[:o[8] + 1 + 2 * nu].copy_(self._dec_bufs[p][0][:o[8] + 1 + 2 * nu], non_blocking=True)
        if n_items:
            self.items_dev[:n_items].copy_(self._items_bufs[p][0][:n_items], non_blocking=True)
        if src is not None:
            # input ids = the in-flight step's sampled tokens, gathered on the device
            if list(src) == list(range(B)):
                self.d_ids[:B].copy_(self.d_out[:B])
            else:
                sb = self._src_bufs[p]
                sb[:B] = torch.as_tensor(src, dtype=torch.int64)
                self.d_src[:B].copy_(sb[:B], non_blocking=True)
                self.d_ids[:B] = self.d_out[self.d_src[:B]]
        return bs

    def _decode_step(self, running: List[_Seq]) -> Tuple[List[_Seq], List[_Seq]]:
        _t0 = time.perf_counter()
        B = len(running)
        lens = np.fromiter((s.length for s in running), dtype=np.int64, count=B)
        last = np.fromiter((s.out[-1] for s in running), dtype=np.int64, count=B)
        bs = self._prep_decode(running, lens, last, 0)
        _t1 = time.perf_counter()
        if self.FAULT_TRIP_DECODE >= 0 and self.steps["decode"] == self.FAULT_TRIP_DECODE \
                and self.par.custom_ar is not None:
            self.par.custom_ar.err.fill_(1)     # fault injection: as if an all-reduce timed out
        self._arm_vote_fault()
        with tracer.gpu_span("engine.decode_forward", bucket=bs, graph=self.use_graphs):
            if self.use_graphs:
                g = self._graphs.get(self._gkey(bs, 0))
                if g is None:
                    g = self._capture(bs, 0)
                g.replay()
            else:
                self._decode_forward(bs, 0)
        self.steps["decode"] += 1
        self.steps["decode_tokens"] += B
        if self.fused_sampler and self.par.custom_ar is not None:
            # tokens and the in-graph health vote of the one-shot all-reduces in ONE read-back
            vals = self.d_out[:bs + 1].tolist()
            if vals[bs]:
                self._collective_trip("decode step")
                self._decode_forward(bs, 0)    # re-run on RCCL: same inputs, idempotent K/V writes
                vals = self.d_out[:bs + 1].tolist()
            toks = vals[:B]
        elif self.fused_sampler:
            toks = self.d_out[:B].tolist()
        else:
            if not self._collectives_ok():
                self._decode_forward(bs, 0)
            toks = self._sample(self.d_hidden[:bs], running, self.d_out[:bs])
        _t2 = time.perf_counter()
        self.timers["decode_host_pre"] += _t1 - _t0
        self.timers["decode_gpu_wait"] += _t2 - _t1
        # stop checks in Python, then ONE native call commits every sequence's K/V and appends
        # the new tokens of those that continue
        eos, mml = self.tok.eos_id, self.max_model_len
        cont = []
        finished: List[_Seq] = []
        for s, t in zip(running, toks):
            t = int(t)
            s.out.append(t)
            p = s.params
            c = not (len(s.out) >= p.max_new_tokens or (not p.ignore_eos and t == eos)
                     or len(s.prompt) + len(s.out) >= mml)
            cont.append(c)
            if not c:
                finished.append(s)
        slots = self.bm.commit_append([s.id for s in running], [s.out[-1] for s in running], cont)
        mb_ = self.max_blocks
        preempted: List[_Seq] = []
        for s, c, slot in zip(running, cont, slots):
            # the appended token sits at position length-1; only a slot that opens a new block
            # (position % BS == 0) can change the row's block table
            if not c or (slot >= 0 and slot % BS != 0):
                continue
            if slot < 0:
                s.error = "__preempt__"
                preempted.append(s)
                continue
            nblk = (s.length + BS - 1) // BS
            blk = slot // BS
            if self.bt_host[s.row, nblk - 1] != blk:
                self.bt_host[s.row, nblk - 1] = blk
                self._bt_upd.extend((s.row * mb_ + nblk - 1, blk))
        self.timers["decode_host_post"] += time.perf_counter() - _t2
        return finished, preempted

    # Pipelined decode (default on the single-GPU graph path): while the GPU runs step k, the host
    # already commits step k's input tokens, reserves the KV slots of the tokens step k is sampling,
    # stages step k+1's inputs and launches it, taking step k's sampled tokens straight from the
    # device (d_out -> d_ids gather); only then does it read step k's tokens back and run the stop
    # checks.  The host work of a step hides under the GPU time of the previous one.  A sequence
    # that stops on EOS at step k has already been launched in step k+1: that one row is computed
    # and discarded (its KV slot belongs to the finished sequence).  Count limits (max_new_tokens,
    # max_model_len) are known in advance and never cost a row.
    PIPELINE = True
    # KV blocks placed in per-sequence runs (csrc/runtime/block_manager.h fresh()): decode attention
    # streams a sequence's blocks in order, and runs read faster than scattered blocks.  0 LIFO,
    # 1 round-5 runs, 2 round-6 runs (in-place continuation, least-held-segment restarts; the default)
    KV_PLACEMENT = 2
    # New requests end a pipelined burst (to be admitted and prefilled) only once the burst has run
    # this many steps: a client that keeps submitting (turn pipelining) would otherwise cut every
    # burst to one or two steps and lose the host/GPU overlap; the added admission delay is at most
    # ADMIT_EVERY decode steps.  1 = admit at the next step (turn-synchronous clients submit only
    # into an idle engine, where it makes no difference).
    ADMIT_EVERY = max(1, int(os.environ.get("DLLM_ADMIT_EVERY", "1")))

    # Tensor-parallel pools pipeline too (class attribute TP_PIPELINE).  Every rank must take the same
    # burst decisions, so a TP burst never looks at the leader-only inbox: it ends on the shared
    # stop rules (tokens, KV blocks and the mirrored waiting list are identical on every rank) or
    # after MIRROR_EVERY steps, when the next admission exchange is due.  The in-graph health vote
    # of the one-shot all-reduces is read back with each step's tokens; a trip ends the burst, the
    # step is re-run on the fallback collectives and the step already in flight is discarded.
    TP_PIPELINE = True

    def _pipeline_ok(self) -> bool:
        return (self.PIPELINE and self.on_gpu and self.use_graphs and self.fused_sampler
                and (not self.par.enabled or self.TP_PIPELINE))

    def _replay(self, bs: int, p: int) -> None:
        if self.FAULT_TRIP_DECODE >= 0 and self.steps["decode"] == self.FAULT_TRIP_DECODE \
                and self.par.custom_ar is not None:
            self.par.custom_ar.err.fill_(1)     # fault injection: as if an all-reduce timed out
        self._arm_vote_fault()
        with tracer.gpu_span("engine.decode_forward", bucket=bs, graph=True):
            g = self._graphs.get(self._gkey(bs, p))
            if g is None:
                g = self._capture(bs, p)
            g.replay()

    def _gkey(self, bs: int, p: int):
        # with step I/O kernels the staging buffer's address is baked into the graph: one graph
        # per bucket and buffer parity
        return (bs, p) if self._gio else bs

    def _read_out(self, B: int, p: int, bs: int) -> "torch.cuda.Event":
        if not self._gio:           # else the step's last kernel (ops.step_store) wrote _out_bufs[p]
            n = bs + 1 if self.par.custom_ar is not None else B    # + the TP health vote at [bs]
            self._out_bufs[p][:n].copy_(self.d_out[:n], non_blocking=True)
        ev = self._out_evts[p]
        ev.record()
        return ev

    # A burst that ends because new requests arrived admits them and queues their prefill chunk
    # BEFORE it waits for its last decode step: the chunk runs right behind that step instead of
    # after the host's admission work (profiles/r4_driver_window_gaps.md: ~2.5 ms of GPU idle per
    # admission).  New sequences only take free rows and free blocks (nothing is released before
    # the burst has drained), and a prefix hit only shares full, committed blocks, never the slot
    # the in-flight step writes.  Single-GPU pools only (TP admissions follow the mirrored schedule).
    EARLY_PREFILL = True

    def _early_admit(self, waiting: List[_Seq], prefilling: Optional[List[_Seq]], running: List[_Seq]) -> None:
        if (prefilling is None or self._early_pf is not None or not self.EARLY_PREFILL or self.par.enabled
                or not self.fused_sampler):
            return
        _t = time.perf_counter()
        adm0 = self.timers["admit"]
        crit = self.host_critical.is_set()
        self.host_critical.set()          # admission host work: in-process clients hold off (bench)
        new = self._take_inbox(final=False)
        self._active.extend(new)          # a failing step must still find them (_abort_all)
        waiting.extend(new)
        # the drain's commit_append runs after this admission: hold back one block for every running
        # row whose next two tokens cross a block boundary (otherwise a just-admitted
        # request can take the block and preempt a running row into a full recompute)
        reserve = sum(1 for s in running if (s.length + 2) // BS != s.length // BS)
        self._admit(waiting, prefilling, len(running), reserve_blocks=reserve)
        if prefilling:
            with tracer.span("engine.prefill_early", "engine", seqs=len(prefilling)):
                self._early_pf = self._prefill_launch(prefilling)
        if not crit:
            self.host_critical.clear()
        self.timers["prefill"] += time.perf_counter() - _t - (self.timers["admit"] - adm0)

    # BURST_JOIN: a pipelined burst no longer ends for admissions.  New requests are admitted and
    # prefilled under the running burst (EARLY_PREFILL), their sequences JOIN the next step once
    # the chunk's first tokens are back, and a finished sequence's blocks and row are released one
    # step after it stopped (when no in-flight step can still write its reserved slot), so rows
    # recycle without a drain.  Needs the step I/O kernels (per-row input ids from the host next to
    # gathered ones); single-GPU pools only.
    BURST_JOIN = True

    def _take_joiners(self, prefilling: List[_Seq], running: List[_Seq], finished: List[_Seq],
                      preempted: List[_Seq]) -> List[_Seq]:
        """Sequences whose early prefill chunk has completed (checked without waiting): their first
        token is appended; those that continue join the next decode step."""
        h = self._early_pf
        if h is None:
            return []
        toks = h[1]
        if isinstance(toks, tuple) and not toks[1].query():
            return []
        _t = time.perf_counter()
        crit = self.host_critical.is_set()
        self.host_critical.set()
        self._early_pf = None
        done = self._prefill_finish(h)
        joiners = []
        for s in done:
            prefilling.remove(s)
            if self._finished(s):     # stopped on its first token: no step ever carries its row
                finished.append(s)
                self._complete_early(s)
                self._release(s)
            elif s.error == "__preempt__":
                preempted.append(s)
            else:
                joiners.append(s)
                running.append(s)
        self.steps["burst_joins"] = self.steps.get("burst_joins", 0) + len(joiners)
        if prefilling and self._early_pf is None:     # chunk budget left some prompts unfinished
            self._early_pf = self._prefill_launch(prefilling)
        if not crit:
            self.host_critical.clear()
        self.timers["prefill"] += time.perf_counter() - _t
        return joiners

    def _decode_burst(self, running: List[_Seq], waiting: List[_Seq],
                      prefilling: Optional[List[_Seq]] = None) -> Tuple[List[_Seq], List[_Seq]]:
        """Pipelined decode steps until the batch must change (a new request arrived, a waiting
        request could take a freed row, or the batch is empty).  Same contract as ``_decode_step``:
        returns (finished, preempted); the caller releases / re-queues them.  On return every
        continuing sequence is in the non-pipelined state (its last token appended with a slot).
        ``prefilling`` (the caller's list): see EARLY_PREFILL."""
        eos, mml, mb_ = self.tok.eos_id, self.max_model_len, self.max_blocks
        finished: List[_Seq] = []
        preempted: List[_Seq] = []
        gone: set = set()           # id(s): finished / preempted inside this burst (rows still in flight are ignored)
        tp = self.par.enabled
        join = (prefilling is not None and self.BURST_JOIN and self._gio and self.EARLY_PREFILL and not tp
                and self._mirror is None and self.fused_sampler)
        self._in_join_burst = join
        release_next: List[_Seq] = []   # stopped in the step just read back: released after the next one
        admit_at = 0                    # step count of the last in-burst admission
        _t0 = time.perf_counter()
        cur = list(running)
        lens = np.fromiter((s.length for s in cur), dtype=np.int64, count=len(cur))
        last = np.fromiter((s.out[-1] for s in cur), dtype=np.int64, count=len(cur))
        pc = 0
        bsk = self._prep_decode(cur, lens, last, pc)
        self._replay(bsk, pc)
        self.host_critical.clear()
        ev = self._read_out(len(cur), pc, bsk)
        vote = self.par.custom_ar is not None     # this step's tokens carry the health vote
        self.steps["decode"] += 1
        nsteps = 1
        self.timers["decode_host_pre"] += time.perf_counter() - _t0
        freed = False               # a row finished while requests wait for one: end the burst
        while True:
            _t0 = time.perf_counter()
            nested0 = self.timers["prefill"] + self.timers["admit"]   # in-burst admission work (own timers)
            alive = [s for s in cur if id(s) not in gone]
            # the next step's rows: sequences that cannot reach a count limit with the token in flight
            nxt = [s for s in alive if len(s.out) + 1 < s.params.max_new_tokens and s.length + 1 < mml]
            joiners = self._take_joiners(prefilling, running, finished, preempted) if join else []
            if join:
                stop = (not nxt and not joiners and self._early_pf is None) or bool(preempted)
            else:
                stop = (not nxt or freed
                        or (nsteps >= self.MIRROR_EVERY if self._mirror is not None
                            else (bool(self._inbox) and nsteps >= self.ADMIT_EVERY))
                        or (bool(waiting) and len(nxt) < len(alive)))
            launched = None
            pending_pre: set = set()
            if stop and joiners:
                # a preemption ends the burst: the joiners' first tokens are appended with slots,
                # so they are plain running sequences for the caller
                joiners = []
            if not stop:
                # commit the in-flight step's input tokens (all alive rows) and reserve the slot of
                # the token each continuing row is sampling right now (placeholder, fixed in post)
                nset = set(map(id, nxt))
                app = [1 if id(s) in nset else 0 for s in alive]
                slots = self.bm.commit_append([s.id for s in alive], [0] * len(alive), app)
                run, src = [], []
                idx = {id(s): i for i, s in enumerate(cur)}
                for s, a, slot in zip(alive, app, slots):
                    if not a:
                        continue
                    if slot < 0:            # out of KV blocks: preempt once its token is known
                        pending_pre.add(id(s))
                        continue
                    if slot % BS == 0:      # the reserved position opens a new block
                        nblk = (s.length + 1 + BS - 1) // BS
                        blk = slot // BS
                        if self.bt_host[s.row, nblk - 1] != blk:
                            self.bt_host[s.row, nblk - 1] = blk
                            self._bt_upd.extend((s.row * mb_ + nblk - 1, blk))
                    run.append(s)
                    src.append(idx[id(s)])
                n_cont = len(run)
                for s in joiners:           # input token known on the host (the chunk's first token)
                    run.append(s)
                    src.append(-1)
                if run:
                    pn = pc ^ 1
                    B = len(run)
                    lens = np.fromiter((s.length + (1 if i < n_cont else 0) for i, s in enumerate(run)),
                                       dtype=np.int64, count=B)
                    last_j = None
                    if joiners:
                        last_j = np.zeros(B, dtype=np.int64)
                        last_j[n_cont:] = [s.out[-1] for s in joiners]
                    bs = self._prep_decode(run, lens, last_j, pn, src=src)
                    self._replay(bs, pn)
                    launched = (run, pn, self._read_out(B, pn, bs), bs, self.par.custom_ar is not None)
                    self.steps["decode"] += 1
                    nsteps += 1
                if (join and (self._inbox or waiting) and self._early_pf is None
                        and nsteps - admit_at >= self.ADMIT_EVERY):
                    admit_at = nsteps
                    self._early_admit(waiting, prefilling, run)
            if launched is None:
                self.host_critical.set()      # until the next burst's first step is launched
                if stop and self._inbox:
                    self._early_admit(waiting, prefilling, [c for c in cur if id(c) not in gone])
            _t1 = time.perf_counter()
            ev.synchronize()
            if self._sync_log is not None:   # diagnostics: how long the loop waited for the step
                self._sync_log.append((_t1 - _t0, time.perf_counter() - _t1, launched is not None))
            if release_next:
                # stopped in the previous read-back: the step that may have carried their row
                # (launched before they were seen to stop) has now completed
                for s in release_next:
                    self._release(s)
                release_next = []
            toks = self._out_np[pc][:len(cur)].tolist()
            tripped = vote and bool(self._out_np[pc][bsk])
            if tripped:
                # a one-shot all-reduce timed out in this step (every rank sees the same vote):
                # discard the step in flight, re-run this one on the fallback collectives, end the burst
                if launched is not None:
                    launched[2].synchronize()
                toks = self._rerun_tripped(cur, pc)
            _t2 = time.perf_counter()
            fix_ids, fix_toks, done_now = [], [], []
            for s, t in zip(cur, toks):
                if id(s) in gone:
                    continue                # a row computed after its sequence stopped
                s.out.append(t)
                self.steps["decode_tokens"] += 1
                pp = s.params
                if (len(s.out) >= pp.max_new_tokens or (not pp.ignore_eos and t == eos)
                        or len(s.prompt) + len(s.out) >= mml):
                    finished.append(s)
                    gone.add(id(s))
                    done_now.append(s)
                elif id(s) in pending_pre:
                    s.error = "__preempt__"
                    preempted.append(s)
                    gone.add(id(s))
                elif launched is not None:
                    fix_ids.append(s.id)
                    fix_toks.append(t)
            if fix_ids:
                self.bm.set_last_tokens(fix_ids, fix_toks)
            if launched is None:
                # drain: the non-pipelined post for the last step (commit its inputs, append the
                # real tokens of the rows that continue)
                rows_ = [s for s in cur if id(s) not in gone or s in done_now]
                cont = [id(s) not in gone for s in rows_]
                slots = self.bm.commit_append([s.id for s in rows_], [s.out[-1] for s in rows_], cont)
                for s, c, slot in zip(rows_, cont, slots):
                    if not c or (slot >= 0 and slot % BS != 0):
                        continue
                    if slot < 0:
                        s.error = "__preempt__"
                        preempted.append(s)
                        continue
                    nblk = (s.length + BS - 1) // BS
                    blk = slot // BS
                    if self.bt_host[s.row, nblk - 1] != blk:
                        self.bt_host[s.row, nblk - 1] = blk
                        self._bt_upd.extend((s.row * mb_ + nblk - 1, blk))
            self.timers["decode_host_pre"] += _t1 - _t0 - (self.timers["prefill"] + self.timers["admit"] - nested0)
            self.timers["decode_gpu_wait"] += _t2 - _t1
            self.timers["decode_host_post"] += time.perf_counter() - _t2
            if launched is None or tripped:
                if tp and self._mirror is not None:
                    self._mirror_iter += nsteps - 1    # admission polls stay ~MIRROR_EVERY steps apart
                self._in_join_burst = False
                return finished, preempted
            if done_now:
                # the next step is already on the GPU: detokenise the stopped answers under it and
                # hand them to their callers now: a short answer must not wait for the
                # longest row of the burst.  Only the KV-block free is deferred to the caller of
                # the burst (the in-flight step may still write the stopped row's reserved slot;
                # nothing allocates blocks before the burst has drained).
                _t3 = time.perf_counter()
                for s in done_now:
                    self._complete_early(s)
                self.timers["complete"] += time.perf_counter() - _t3
                if join:
                    release_next.extend(done_now)
            freed = bool(waiting) and bool(done_now or preempted)
            cur, pc, ev, bsk, vote = launched

    def _rerun_tripped(self, cur: List[_Seq], p: int) -> List[int]:
        """Pipelined TP step whose health vote tripped: drop the one-shot all-reduce and re-run the
        step eagerly on the fallback collectives.  Its inputs are rebuilt from the host state (the
        previous step's tokens are already appended), its K/V writes are idempotent."""
        self._collective_trip("decode step")
        B = len(cur)
        lens = np.fromiter((s.length for s in cur), dtype=np.int64, count=B)
        last = np.fromiter((s.out[-1] for s in cur), dtype=np.int64, count=B)
        bs = self._prep_decode(cur, lens, last, p)
        self._decode_forward(bs, p)
        return self.d_out[:B].tolist()

    def _complete_early(self, s: _Seq) -> None:
        """A sequence stopped inside a pipelined burst: record its finish time, form its text and
        wake its caller; ``_release`` (after the burst) frees its blocks and row."""
        s.finished = time.perf_counter()
        self._finalize_text(s)
        s.finish()

    # fault injection (tests): force a collective trip on the Nth decode / prefill step of every rank
    FAULT_TRIP_DECODE = fault("car_trip_decode", -1, int)
    FAULT_TRIP_PREFILL = fault("car_trip_prefill", -1, int)

    # fault injection (tests): on decode step FAULT_VOTE_DECODE, rank FAULT_VOTE_RANK's one-shot
    # all-reduce flag is raised DURING the in-graph health vote (after its vote was staged)
    FAULT_VOTE_DECODE = fault("car_vote_decode", -1, int)
    FAULT_VOTE_RANK = fault("car_vote_rank", 0, int)

    def _arm_vote_fault(self) -> None:
        car = self.par.custom_ar
        if car is None or self.FAULT_VOTE_DECODE < 0:
            return
        if getattr(car, "fault_vote", None) is None:
            car.fault_vote = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._graphs.clear()     # re-captured with the injection op
        # fires once, on the first step replayed at or after FAULT_VOTE_DECODE (a pipelined burst
        # counts its steps when they are read back, after later steps were already issued)
        hit = (self.steps["decode"] >= self.FAULT_VOTE_DECODE and not getattr(self, "_vote_fault_fired", False)
               and self.par.tp_rank == self.FAULT_VOTE_RANK)
        if hit:
            self._vote_fault_fired = True
            self.vote_fault_step = self.steps["decode"]
        car.fault_vote.fill_(1 if hit else 0)

    def _collective_trip(self, where: str) -> None:
        """Every TP rank sees the same trip on the same step: drop the one-shot all-reduce (its
        epochs are out of step), drop the graphs that embed it (re-captured on demand), and let
        the caller re-run the step on RCCL."""
        self.par.drop_custom_ar(f"timed out on a peer during a {where}")
        self._graphs.clear()
        self._check_graph_collectives()
        self.collective_trips = getattr(self, "collective_trips", 0) + 1
        self.trip_steps.append(self.steps["decode"])

    # Tensor-parallel decode graphs (on by default; DLLM_TP_GRAPHS=0 decodes TP pools eagerly).  A
    # replay fault seen early in round 3 on the one-GPU TP=2 rehearsal came from torch.topk's
    # multi-block select inside the captured step; with the vocab-parallel sampler on its own kernels
    # (ops.tp_candidates / ops.tp_sample) TP=2/4 graphs replay clean across prefills, graph/eager
    # alternation and an injected collective trip (profiles/r3_tp_graph_fault.md,
    # profiles/r3_multirank_one_gpu.md), and TP=4 decode runs 23 % faster than eager there.
    TP_GRAPHS = os.environ.get("DLLM_TP_GRAPHS", "1") == "1"

    def _check_graph_collectives(self) -> None:
        """A TP decode graph can only capture device collectives: the one-shot IPC kernels or RCCL.
        A group on gloo (one-GPU multi-process tests) without the one-shot all-reduce runs eager;
        so does every TP group unless ``TP_GRAPHS``."""
        if not self.par.enabled or not self.use_graphs:
            return
        if not self.TP_GRAPHS:
            self.use_graphs = False
            return
        if self.par.custom_ar is not None:
            return
        import torch.distributed as dist
        if self.par.tp_group is None or dist.get_backend(self.par.tp_group) != "nccl":
            self.use_graphs = False

    def _collectives_ok(self) -> bool:
        """Prefill / unfused-sampler steps: MAX-reduce the one-shot all-reduce's error flag over
        the group (one small collective + host read); False = the caller re-runs the step."""
        if self.par.custom_ar is None:
            return True
        if self.FAULT_TRIP_PREFILL >= 0 and self.steps["prefill"] == self.FAULT_TRIP_PREFILL:
            self.par.custom_ar.err.fill_(1)
        if self.par.check_collectives():
            return True
        self._graphs.clear()
        self._check_graph_collectives()
        self.collective_trips = getattr(self, "collective_trips", 0) + 1
        return False

    def _decode_meta(self, bs: int) -> AttnMeta:
        if self._use_worklist(bs):
            return AttnMeta(slots=self.d_slots[:bs], block_tables=self.bt_dev, qstart=self.d_qstart,
                            qlen=self.d_qlen, ctx=self.d_ctx, tile_seq=self.d_tseq[:bs], tile_tok0=self.d_tok0[:bs],
                            last_idx=self.d_last[:bs], all_last=True, splits=self.max_splits, workspace=self.dec_ws,
                            items=self.items_dev, grid_items=self._attn_grid(bs))
        return AttnMeta(slots=self.d_slots[:bs], block_tables=self.bt_dev, qstart=self.d_qstart, qlen=self.d_qlen,
                        ctx=self.d_ctx, tile_seq=self.d_tseq[:bs], tile_tok0=self.d_tok0[:bs],
                        last_idx=self.d_last[:bs], all_last=True, splits=self._decode_splits(bs), workspace=self.dec_ws,
                        split_len=self.d_split if self.ATTN_DYNAMIC else None)

    def _decode_forward(self, bs: int, p: int = 0) -> None:
        with ops.gemm.workspace_owner(self._ws_owner):
            self._decode_forward_inner(bs, p)

    def _decode_forward_inner(self, bs: int, p: int = 0) -> None:
        if self._gio:
            o, mb = self._off, self.buckets[-1]
            items = (self._items_bufs[p][0], self.items_dev) if self.attn_worklist else (None, None)
            ops.step_fetch(self._dec_bufs[p][0], self.dec_dev, o[0], o[9], mb, self.d_out, *items)
        self._decode_body(bs)
        if self._gio:
            ops.step_store(self.d_out, self._out_bufs[p], bs + 1)

    def _decode_body(self, bs: int) -> None:
        # this step's block-table updates (inside the graph; the fused layer applies them in its
        # embedding launch)
        hid = self.model.hidden_states(self.d_ids[:bs], self.d_pos[:bs], self._decode_meta(bs), self.kv_caches,
                                       scatter=(self.bt_dev, self.d_upd))
        if self.fused_sampler:
            self.model.sample(hid, self.d_temp[:bs], self.d_topp[:bs], self.d_topk[:bs], self.d_seed,
                              self.d_out[:bs])
            if self.par.custom_ar is not None:
                self.par.graph_error_flag(self.d_out[bs:bs + 1])
            return
        self.d_hidden[:bs].copy_(hid)
        self.d_out[:bs].copy_(self.model.greedy(hid))

    def _capture(self, bs: int, p: int = 0) -> "torch.cuda.CUDAGraph":
        # warm up (lazy library init must not happen inside capture), then capture.  A graph
        # captured lazily mid-burst warms up on the real step: with the id gather inside the step
        # (step I/O kernels) the warm-up's sampler would overwrite the previous step's tokens the
        # replay gathers its input ids from, so d_out is restored after it.
        saved = self.d_out.clone() if self._gio else None
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._decode_forward(bs, p)
        torch.cuda.current_stream(self.device).wait_stream(s)
        if saved is not None:
            self.d_out.copy_(saved)
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self._graph_pool):
            self._decode_forward(bs, p)
        self._graphs[self._gkey(bs, p)] = g
        return g

    def capture_all(self, max_bs: Optional[int] = None) -> None:
        """Pre-capture decode graphs for every bucket up to ``max_bs`` (largest first)."""
        if not self.use_graphs:
            return
        # a dummy decode state in both staging buffers: all padding (qlen 0), so the warm-up runs
        # of the captures write nothing to the KV cache
        o, mb = self._off, self.buckets[-1]
        for _, h, _ in self._dec_bufs:
            h[:] = 0
            h[o[2]:o[3]] = -1
            h[o[3]:o[4]] = self.R
            h[o[9]:o[9] + mb] = -1
        if self.attn_worklist:
            for _, it in self._items_bufs:
                it[:4] = 0
        self.dec_dev.copy_(self.dec_host_t)
        self._sync_bt()
        for b in sorted((b for b in self.buckets if max_bs is None or b <= max_bs), reverse=True):
            for p in ((0, 1) if self._gio else (0,)):
                if self._gkey(b, p) not in self._graphs:
                    self._capture(b, p)
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ outputs
    def _finalize_text(self, s: _Seq) -> str:
        """Detokenise a stopped sequence's answer and memoise prompt+answer ids for the next turn.

        Called from the decode loop the moment a sequence stops (``_decode_burst``), so with
        pipelined decode this host work runs while the GPU executes the next step instead of in
        one serial pass after the whole batch has finished; ``_output`` re-uses the result."""
        if s.out_text is not None:
            return s.out_text
        toks = [t for t in s.out if t != self.tok.eos_id] if not s.params.ignore_eos else list(s.out)
        # strip whitespace-only tokens at both ends so that text == decode(ids) exactly (pools strip)
        while toks and not self.tok.decode(toks[:1]).strip():
            toks.pop(0)
        while toks and not self.tok.decode(toks[-1:]).strip():
            toks.pop()
        text = self.tok.decode(toks)
        if s.text is not None and s.error is None and text:
            self._remember(s.text + text, s.prompt + toks)
        s.out_text = text
        return text

    def _output(self, s: _Seq) -> RequestOutput:
        end = s.finished or time.perf_counter()
        lat = (end - s.arrival) * 1000.0
        ttft = ((s.first_tok or end) - s.arrival) * 1000.0
        queue = ((s.admitted or end) - s.arrival) * 1000.0
        n = len(s.out)
        dec_t = (end - s.first_tok) if s.first_tok else 0.0
        text = self._finalize_text(s)
        return RequestOutput(s.id, text, list(s.out), len(s.prompt), s.num_cached, n, lat, ttft,
                             queue, (n - 1) / dec_t if n > 1 and dec_t > 0 else 0.0, s.error)
