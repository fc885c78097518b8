"""One-shot all-reduce over IPC-mapped peer buffers (xGMI) for decode-size TP messages.

SURVEY §2.7 / §5.8: decode-time tensor-parallel all-reduces are B x H bf16 (8-16 KiB x B),
latency-bound; a ring all-reduce pays 2(w-1) hops on the per-link-bound xGMI mesh, whereas every
MI355X in a node has a direct link to every other one.  ``CustomAllReduce`` maps every TP peer's
buffer into this process (hipIpcGetMemHandle / hipIpcOpenMemHandle), and one kernel
(csrc/kernels/custom_ar.hip) copies, flags, reads all peers and sums — no host sync, so it runs
inside the captured decode hipGraph.  Messages above ``max_bytes`` (prefill) go to RCCL.

The reference has no collectives at all (HTTP RPC only, reference src/router.py:152-171); this is
the MI355X-native data plane the survey plans for the large pool.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

DEFAULT_MAX_BYTES = int(os.environ.get("DLLM_CUSTOM_AR_MAX_BYTES", str(1 << 20)))


def _ext():
    from .. import ops
    k = ops._load()
    if k is None:
        raise ops.NativeOpsMissing(f"custom all-reduce needs the HIP extension ({ops._ext_err})")
    return k


class CustomAllReduceUnavailable(RuntimeError):
    pass


class CustomAllReduce:
    """Per-TP-group communicator.  Every rank of ``group`` must construct it (collective)."""

    def __init__(self, group, device: torch.device, max_bytes: int = DEFAULT_MAX_BYTES,
                 spin_limit: int = 1 << 22):
        self.group = group
        self.device = torch.device(device)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("one-shot all-reduce supports at most 8 ranks (one xGMI hop)")
        self.max_bytes = (max_bytes + 15) // 16 * 16
        self.spin_limit = spin_limit
        k = _ext()
        # every step is agreed on by the whole group, so a rank whose IPC setup fails makes ALL
        # ranks fall back to RCCL together (a one-sided fallback would deadlock the collective)
        self._base, self._opened = 0, []
        handle, err = None, None
        try:
            with torch.cuda.device(self.device):
                self._base = k.car_alloc(self.max_bytes)
                handle = k.car_handle(self._base)
                torch.cuda.synchronize(self.device)
        except Exception as e:  # noqa: BLE001 - reported to every rank below
            err = f"rank {self.rank}: {e}"
        got: List[Optional[tuple]] = [None] * self.world
        dist.all_gather_object(got, (handle, err), group=group)
        errs = [g[1] for g in got if g[1]]
        if errs:
            self.close()
            raise CustomAllReduceUnavailable("; ".join(errs))
        bases, err = [], None
        try:
            with torch.cuda.device(self.device):
                for p, (h, _) in enumerate(got):
                    if p == self.rank:
                        bases.append(self._base)
                    else:
                        ptr = k.car_open(h)
                        self._opened.append(ptr)
                        bases.append(ptr)
        except Exception as e:  # noqa: BLE001
            err = f"rank {self.rank}: {e}"
        oks: List[Optional[str]] = [None] * self.world
        dist.all_gather_object(oks, err, group=group)
        errs = [e for e in oks if e]
        if errs:
            self.close()
            raise CustomAllReduceUnavailable("; ".join(errs))
        self.bases = bases
        self.counters = torch.zeros(2, dtype=torch.int32, device=self.device)
        # [0]: sticky timeout flag (bit per peer), [1]: its snapshot when the health vote is staged
        self.err = torch.zeros(2, dtype=torch.int32, device=self.device)
        self.flag_vec = torch.zeros(8, dtype=torch.bfloat16, device=self.device)   # in-graph health vote
        dist.barrier(group=group)  # every region zeroed + mapped before the first flag is written
        self.calls = 0

    def eligible(self, t: torch.Tensor) -> bool:
        n = t.numel() * t.element_size()
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and n % 16 == 0
                and 0 < n <= self.max_bytes)

    def vote_stage(self, v: torch.Tensor) -> None:
        """Health vote, before its all-reduce: v[:8] = (this rank's error flag != 0, 0, ...), and
        the flag's snapshot in err[1]."""
        _ext().car_vote(0, self.err, v, self.err)

    def vote_decide(self, v: torch.Tensor, out: torch.Tensor) -> None:
        """Health vote, after its all-reduce: out[0] = 1 if this rank voted 1 or a peer did; a flag
        raised only by the vote's own all-reduce defers the trip to the next step's vote (the
        kernel's comment in custom_ar.hip has the agreement argument)."""
        _ext().car_vote(1, self.err, v, out)

    def all_reduce(self, t: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Sum ``t`` over the group into ``out`` (default: in place).  Caller checks eligible()."""
        out = t if out is None else out
        _ext().car_allreduce(t, out, self.bases, self.rank, self.max_bytes, self.counters, self.err,
                             self.spin_limit)
        self.calls += 1
        return out

    def resadd_slots(self, H: int) -> int:
        return int(_ext().car_resadd_slots(int(H)))

    def eligible_resadd(self, y: torch.Tensor, r: torch.Tensor) -> bool:
        return (self.eligible(y) and y.dim() == 2 and r.dtype == torch.bfloat16 and r.stride(1) == 1
                and r.stride(0) % 8 == 0 and self.resadd_slots(y.shape[1]) >= 1)

    def all_reduce_resadd(self, y: torch.Tensor, r: torch.Tensor, ssq: torch.Tensor, add: bool = True) -> int:
        """``r += sum_p y_p`` (``r = sum`` when not ``add``) in place with the new r's partial row
        sums of squares in ``ssq[:slots]``; one launch (csrc/kernels/custom_ar.hip car_resadd_kernel).
        Returns the slot count."""
        n = _ext().car_resadd(y, r, ssq, bool(add), self.bases, self.rank, self.max_bytes, self.counters, self.err,
                              self.spin_limit)
        self.calls += 1
        return int(n)

    def eligible_gather(self, t: torch.Tensor) -> bool:
        n = t.numel() * t.element_size()
        return t.is_cuda and t.is_contiguous() and n % 16 == 0 and 0 < n <= self.max_bytes

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape] of every rank's ``t`` (one launch, graph-capturable)."""
        out = torch.empty((self.world, *t.shape), dtype=t.dtype, device=t.device)
        _ext().car_allgather(t, out, self.bases, self.rank, self.max_bytes, self.counters, self.err, self.spin_limit)
        self.calls += 1
        return out

    def check(self) -> None:
        """Raise if any call timed out waiting for a peer (bitmask of missing peers)."""
        e = int(self.err[0].item())
        if e:
            raise RuntimeError(f"custom all-reduce: peer flags never arrived (mask {e:#x}); "
                               "TP ranks are out of step")

    def close(self) -> None:
        if not self._base and not self._opened:
            return
        k = _ext()
        for p in self._opened:
            k.car_close(p)
        self._opened = []
        if self._base:
            k.car_free(self._base)
            self._base = 0
