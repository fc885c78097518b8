"""Expert parallelism for the MoE large tier (Mixtral-8x7B): all-to-all dispatch + combine.

SURVEY §2.5 lists "EP all-to-all (optional MoE expert-parallel) — [tokens·2, H] dispatch +
combine, 2 per MoE layer"; the reference itself has no collectives (it delegates to Ollama).

MI355X-first layout.  The default MoE sharding is TP-within-expert (every rank holds 1/P of every
expert's intermediate dim, one all-reduce per layer, graph-capturable).  EP mode instead gives
each rank E/P WHOLE experts, so an expert's weights are streamed by exactly one GPU and each
grouped GEMM sees P x more rows — the better trade for prefill-sized batches, where TP-within-
expert runs P skinny GEMMs per expert.  Activations after the TP attention all-reduce are
replicated across the group, so each rank owns a 1/P slice of the tokens (sequence-parallel
style), and one MoE layer is:

  gate (local slice)  ->  all-to-all #1: token rows + local expert id to the expert's owner
  grouped expert FFN on the received rows (ops.moe_ffn: HIP gate/permute/grouped MFMA GEMMs)
  all-to-all #2: expert outputs back to the token's owner -> weighted combine (fp32 index_add)
  all-gather: every rank gets the full [T, H] MoE output again (replicated for the next layer)

Split sizes travel first as a tiny all-to-all of counts, so only real rows move (no capacity
padding, no dropped tokens); that count exchange is a host sync, so EP runs the prefill-size
batches only (``LlamaModel.use_ep``: >= DLLM_EP_MIN_TOKENS tokens, eager).  Decode steps run the
TP-within-expert shards that an EP model keeps resident as well, so they stay graph-captured
(memory for latency: Mixtral TP=8 holds 11.6 GB more per GPU of a 288 GB part).  Over xGMI every all-to-all is
P-1 point-to-point transfers on distinct links, which is the pattern the fully connected
MI355X mesh serves best (no ring hops).
"""
from __future__ import annotations

from typing import List, Tuple

import torch
import torch.distributed as dist

from .. import ops


def token_slice(T: int, rank: int, size: int) -> Tuple[int, int]:
    """This rank's contiguous token range of a replicated [T, H] batch (uneven T allowed)."""
    base, extra = divmod(T, size)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _staged(t: torch.Tensor, group) -> bool:
    """Device tensors on a gloo group (CPU tests' groups, the one-GPU multi-process rehearsal) go
    through the host: gloo's all-to-all / all-gather take CPU tensors."""
    return t.is_cuda and dist.get_backend(group) != "nccl"


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits: List[int], in_splits: List[int], group) -> None:
    if _staged(out, group):
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.contiguous().cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
        return
    dist.all_to_all_single(out, inp.contiguous(), out_splits, in_splits, group=group)


def ep_moe_ffn(x: torch.Tensor, ids: torch.Tensor, wts: torch.Tensor, w13_local: torch.Tensor,
               w2_local: torch.Tensor, n_experts: int, group, size: int) -> torch.Tensor:
    """MoE FFN of this rank's tokens with experts sharded over ``group`` (E/size per rank).

    x [T, H] (this rank's tokens), ids [T, k] global expert ids, wts [T, k] f32 combine weights,
    w13_local [E/size, 2I, H], w2_local [E/size, H, I] (this rank's experts).  Returns [T, H].
    Every rank of ``group`` must call this for the same layer (the all-to-alls are collective),
    with T = 0 allowed.
    """
    T, H = x.shape
    k = ids.shape[1] if ids.dim() == 2 else 1
    e_loc = n_experts // size
    dev = x.device
    tok = torch.arange(T, device=dev).repeat_interleave(k)
    eid = ids.reshape(-1).long()
    wt = wts.reshape(-1).float()
    dest = eid // e_loc
    order = torch.argsort(dest, stable=True)
    tok, eid, wt, dest = tok[order], eid[order], wt[order], dest[order]
    send_counts = torch.bincount(dest, minlength=size).to(torch.int64)
    recv_counts = torch.empty_like(send_counts)
    _a2a(recv_counts, send_counts, None, None, group)
    ss, rs = send_counts.tolist(), recv_counts.tolist()
    n_recv = sum(rs)
    recv_x = torch.empty((n_recv, H), dtype=x.dtype, device=dev)
    _a2a(recv_x, x.index_select(0, tok), rs, ss, group)
    recv_e = torch.empty(n_recv, dtype=torch.int32, device=dev)
    _a2a(recv_e, (eid % e_loc).to(torch.int32), rs, ss, group)
    if n_recv:
        # every received row is one (token, expert) pair: top-1 routing with weight 1 locally
        y = ops.moe_ffn(recv_x, recv_e.view(-1, 1), torch.ones((n_recv, 1), dtype=torch.float32, device=dev),
                        w13_local, w2_local)
    else:
        y = recv_x
    back = torch.empty((tok.numel(), H), dtype=x.dtype, device=dev)
    _a2a(back, y, ss, rs, group)
    out = torch.zeros((T, H), dtype=torch.float32, device=dev)
    out.index_add_(0, tok, back.float() * wt.unsqueeze(1))
    return out.to(x.dtype)


def all_gather_rows(x_local: torch.Tensor, T: int, group, size: int) -> torch.Tensor:
    """Inverse of :func:`token_slice`: concatenate every rank's rows into the full [T, H]."""
    sizes = [token_slice(T, r, size) for r in range(size)]
    mx = max(hi - lo for lo, hi in sizes)
    H = x_local.shape[1]
    pad = torch.zeros((mx, H), dtype=x_local.dtype, device=x_local.device)
    pad[:x_local.shape[0]] = x_local
    if x_local.is_cuda and not _staged(x_local, group):
        buf = torch.empty((size, mx, H), dtype=x_local.dtype, device=x_local.device)
        dist.all_gather_into_tensor(buf, pad, group=group)
        parts = [buf[r, :hi - lo] for r, (lo, hi) in enumerate(sizes)]
    else:
        src = pad.cpu()
        bufs = [torch.empty_like(src) for _ in range(size)]
        dist.all_gather(bufs, src, group=group)
        parts = [bufs[r][:hi - lo] for r, (lo, hi) in enumerate(sizes)]
    return torch.cat(parts, 0).to(x_local.device)
