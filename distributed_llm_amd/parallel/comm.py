"""Process groups and collectives (RCCL over xGMI on MI355X; gloo on CPU for tests).

One process per GPU (``torch.distributed``, backend "nccl" == RCCL on ROCm).  A node is
partitioned into *pools*: each pool is a contiguous rank range with its own tensor-parallel
group (e.g. 8 GPUs = small pool ranks 0-1 as two TP=1 replicas + large pool ranks 4-7 as one
TP=4 group).  Collectives used on the serving path:
  * TP all-reduce after o_proj / down_proj (decode messages are B x H bf16 = 8-16 KiB x B,
    latency-bound — kept as ONE call per sub-layer, never split);
  * vocab-parallel LM head: all-gather of per-rank (max, argmax) pairs or per-rank top-k
    candidates instead of the full [B, V] logits;
  * point-to-point send/recv between pools (failover hand-off, health probes) — parallel.p2p.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


@dataclass
class ParallelContext:
    tp_size: int = 1
    tp_rank: int = 0
    tp_group: Optional[object] = None   # torch ProcessGroup
    global_rank: int = 0
    world_size: int = 1
    custom_ar: Optional[object] = None  # parallel.custom_ar.CustomAllReduce (GPU TP groups)
    moe_ep: bool = False                # MoE layers expert-parallel over the TP group (parallel.expert_parallel)
    # Megatron-style sequence parallelism for prefill-size batches under TP: the residual stream
    # and the norms run on a 1/tp token shard (reduce-scatter + all-gather replace each all-reduce)
    sequence_parallel: bool = field(default_factory=lambda: os.environ.get("DLLM_SEQ_PARALLEL", "0") == "1")
    sp_min_tokens: int = field(default_factory=lambda: int(os.environ.get("DLLM_SP_MIN_TOKENS", "256")))
    sp_calls: int = 0                   # sequence-parallel reductions run (tests: SP really ran)

    @property
    def enabled(self) -> bool:
        return self.tp_size > 1

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the TP group: one-shot xGMI kernel for decode-size bf16 messages,
        RCCL for everything else (prefill activations, f32, CPU/gloo)."""
        if self.tp_size > 1:
            car = self.custom_ar
            if car is not None and car.eligible(t):
                car.all_reduce(t)
            else:
                self._group_all_reduce(t)
        return t

    def _group_all_reduce(self, t: torch.Tensor) -> None:
        """RCCL, or gloo (CPU tests, the one-GPU multi-process rehearsal): device tensors are
        staged through the host there, so the fallback after a one-shot all-reduce trip never
        depends on gloo's device support."""
        if t.is_cuda and dist.get_backend(self.tp_group) != "nccl":
            h = t.cpu()
            dist.all_reduce(h, group=self.tp_group)
            t.copy_(h)
        else:
            dist.all_reduce(t, group=self.tp_group)

    def all_reduce_resadd(self, y: torch.Tensor, r: torch.Tensor, ssq: torch.Tensor, add: bool = True) -> int:
        """Row-parallel output epilogue of the fused tensor-parallel layer: ``r += sum over the TP
        group of y`` (``r = sum`` when not ``add``: the vocab-parallel embedding) in place, plus the
        new residual's partial row sums of squares in ``ssq`` for the next fused RMSNorm-folding
        GEMM.  One kernel when the one-shot all-reduce takes the message (decode), else RCCL
        all-reduce + the res_add_ssq kernel.  Returns the number of ssq slots written."""
        from .. import ops
        car = self.custom_ar
        if self.tp_size > 1 and car is not None and car.eligible_resadd(y, r):
            return car.all_reduce_resadd(y, r, ssq, add)
        if self.tp_size > 1:
            self._group_all_reduce(y)
        if add:
            return ops.gemm.res_add_ssq(y, r, ssq)
        r.copy_(y)
        return ops.gemm.res_add_ssq(None, r, ssq)

    def sp_resadd(self, y: torch.Tensor, r: torch.Tensor, ssq: torch.Tensor) -> int:
        """Sequence-parallel form of :meth:`all_reduce_resadd` for prefill-size batches of the
        fused layer (Megatron-SP): the row-parallel partial sums are reduce-scattered to this
        rank's token slice, the residual add runs on the slice only, and the updated slices are
        all-gathered back into the replicated residual ``r`` that the next column-parallel fused
        GEMM reads (its RMSNorm row statistics are recomputed from the gathered rows: every rank
        holds the same r, so the statistics are bitwise equal).  Same bytes on the wire as one
        all-reduce; the add and the [T, H] reduction output shrink by tp."""
        from .. import ops
        from .expert_parallel import token_slice
        T = y.shape[0]
        lo, hi = token_slice(T, self.tp_rank, self.tp_size)
        ys = self.reduce_scatter_rows(y)
        rs = r[lo:hi]
        if hi > lo:
            ops.gemm.res_add_ssq(ys, rs, torch.empty(hi - lo, dtype=torch.float32, device=r.device))
        r.copy_(self.all_gather_rows(rs, T))
        self.sp_calls += 1
        return ops.gemm.res_add_ssq(None, r, ssq)

    def enable_custom_all_reduce(self, device, max_bytes: Optional[int] = None) -> bool:
        """Collective over the TP group.  Returns False (RCCL only) when not applicable."""
        if self.tp_size <= 1 or self.tp_size > 8 or torch.device(device).type != "cuda":
            return False
        if os.environ.get("DLLM_CUSTOM_AR", "1") == "0":
            return False
        from .custom_ar import DEFAULT_MAX_BYTES, CustomAllReduce, CustomAllReduceUnavailable
        try:
            self.custom_ar = CustomAllReduce(self.tp_group, torch.device(device), max_bytes or DEFAULT_MAX_BYTES)
        except CustomAllReduceUnavailable as e:  # agreed by every rank: all stay on RCCL
            import logging
            logging.getLogger(__name__).warning("custom all-reduce disabled: %s", e)
            return False
        return True

    def graph_error_flag(self, out: torch.Tensor) -> None:
        """In-graph health vote of the one-shot all-reduce, appended to a decode step: every rank
        contributes (its error flag != 0) to one more 16-byte one-shot all-reduce and writes
        ``sum > 0 or own flag`` into ``out`` (an int32 slot read back WITH the step's tokens), so
        live ranks agree on a trip without a per-step host all-reduce: a rank that timed out on a
        peer during the step votes 1 and trips, and every rank that completes the vote sees that
        1; a rank whose flag was raised only by the vote's own all-reduce does NOT trip alone (its
        step data was clean) but carries the sticky flag into the next step's vote, so every rank
        trips on the same later step (a lone re-run would pair RCCL calls of different
        steps across ranks)."""
        car = self.custom_ar
        if car is None:
            out.zero_()
            return
        v = car.flag_vec
        car.vote_stage(v)          # v = (err != 0, 0, ...), err[1] = snapshot: one launch
        fault = getattr(car, "fault_vote", None)
        if fault is not None:      # fault injection (tests): a timeout raised DURING the vote
            car.err[:1].bitwise_or_(fault)
        car.all_reduce(v)
        car.vote_decide(v, out)    # out = own snapshot | (vote completed and sum > 0): one launch

    def drop_custom_ar(self, why: str) -> None:
        """Every rank of the group calls this on the same step (agreed trip): RCCL carries every
        later all-reduce; the one-shot buffers stay mapped until process exit."""
        import logging
        logging.getLogger(__name__).error("custom all-reduce dropped: %s; continuing on RCCL", why)
        self.custom_ar = None

    def check_collectives(self) -> bool:
        """After a step: did any rank's one-shot all-reduce time out waiting for a peer (its error
        flag, parallel.custom_ar)?  The flag is MAX-reduced over the TP group so every rank takes
        the same decision; on a trip the custom all-reduce is dropped on ALL ranks (its epochs are
        out of step from then on) and RCCL carries every later all-reduce.  Returns False on a
        trip — the caller must discard the step (its sums may hold stale peer data)."""
        car = self.custom_ar
        if car is None:
            return True
        flag = car.err.detach().clone()
        if self.tp_group is not None and dist.is_initialized():
            if dist.get_backend(self.tp_group) != "nccl":
                flag = flag.cpu()
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.tp_group)
        if int(flag.reshape(-1)[0].item()) == 0:
            return True
        import logging
        logging.getLogger(__name__).error("custom all-reduce timed out (peer mask %#x): falling back to RCCL",
                                          int(flag.reshape(-1)[0].item()))
        self.custom_ar = None
        return False

    def use_sp(self, num_tokens: int) -> bool:
        return self.sequence_parallel and self.tp_size > 1 and num_tokens >= max(self.sp_min_tokens, self.tp_size)

    def reduce_scatter_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Sum [T, H] partial activations over the TP group and keep this rank's token slice
        (``expert_parallel.token_slice`` layout, uneven T allowed): half the bytes of an
        all-reduce leave each rank, the other half return in the matching all-gather."""
        from .expert_parallel import token_slice
        T = t.shape[0]
        lo, hi = token_slice(T, self.tp_rank, self.tp_size)
        if not t.is_cuda or dist.get_backend(self.tp_group) != "nccl":
            # gloo has no reduce-scatter: all-reduce (host-staged for device tensors: the one-GPU
            # multi-process rehearsal) and slice
            self._group_all_reduce(t)
            return t[lo:hi].contiguous()
        mx = -(-T // self.tp_size)
        buf = torch.zeros((self.tp_size, mx, *t.shape[1:]), dtype=t.dtype, device=t.device)
        for r in range(self.tp_size):
            a, b = token_slice(T, r, self.tp_size)
            buf[r, :b - a] = t[a:b]
        out = torch.empty((mx, *t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(out, buf.view(-1, *t.shape[1:]), group=self.tp_group)
        return out[:hi - lo]

    def all_gather_rows(self, t: torch.Tensor, T: int) -> torch.Tensor:
        from .expert_parallel import all_gather_rows
        return all_gather_rows(t.contiguous(), T, self.tp_group, self.tp_size)

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenate ``t`` from every TP rank along a new leading dim -> [tp, *t.shape]."""
        if self.tp_size == 1:
            return t.unsqueeze(0)
        t = t.contiguous()
        car = self.custom_ar
        if car is not None and car.eligible_gather(t):   # one-shot IPC gather (decode candidates)
            return car.all_gather(t)
        if t.is_cuda and dist.get_backend(self.tp_group) == "nccl":  # RCCL: one fused all-gather
            out = torch.empty((self.tp_size, *t.shape), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t, group=self.tp_group)
            return out
        # gloo (CPU tests, one-GPU rehearsal): stage device tensors through the host
        src = t.cpu() if t.is_cuda else t
        parts = [torch.empty_like(src) for _ in range(self.tp_size)]
        dist.all_gather(parts, src, group=self.tp_group)
        out = torch.stack(parts)
        return out.to(t.device) if t.is_cuda else out


SINGLE = ParallelContext()


def init_distributed(backend: Optional[str] = None) -> ParallelContext:
    """Initialise the default process group from torchrun env vars (idempotent)."""
    if not dist.is_available():
        return SINGLE
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and not dist.is_initialized():
        return SINGLE
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group(backend=backend)
    r, w = dist.get_rank(), dist.get_world_size()
    return ParallelContext(tp_size=1, tp_rank=0, tp_group=None, global_rank=r, world_size=w)


def make_tp_groups(tp: int, ranks: Optional[Sequence[int]] = None) -> ParallelContext:
    """Split ``ranks`` (default: all) into consecutive TP groups of size ``tp``.

    Every rank must call this with the same arguments (new_group is collective).
    Returns this rank's context (tp_size 1 if the rank is not in ``ranks``).
    """
    if not dist.is_initialized():
        if tp != 1:
            raise RuntimeError("tensor parallelism needs torch.distributed initialised")
        return SINGLE
    world, me = dist.get_world_size(), dist.get_rank()
    ranks = list(range(world)) if ranks is None else list(ranks)
    if len(ranks) % tp != 0:
        raise ValueError(f"{len(ranks)} ranks not divisible by tp={tp}")
    mine = ParallelContext(1, 0, None, me, world)
    for i in range(0, len(ranks), tp):
        grp_ranks = ranks[i:i + tp]
        g = dist.new_group(grp_ranks) if tp > 1 else None
        if me in grp_ranks:
            mine = ParallelContext(tp, grp_ranks.index(me), g, me, world)
    return mine


def shard_range(n: int, rank: int, size: int) -> slice:
    if n % size != 0:
        raise ValueError(f"dimension {n} not divisible by tp={size}")
    k = n // size
    return slice(rank * k, (rank + 1) * k)
