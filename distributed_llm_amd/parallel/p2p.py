"""Point-to-point messaging between pools (RCCL send/recv over xGMI on GPU ranks; gloo on CPU).

Control messages between the router and a pool leader travel on a CPU (gloo) group with tags
(pools.remote: request tag 1, reply tag 2; many requests in flight); the RCCL pair group is the
data plane (token ids, pings).

The reference moves every request as HTTP/JSON through an SSH tunnel to a remote board
(src/models/nano.py:23-35) and re-sends the full history on failover (src/router.py:277-282).
On one MI355X node, pools are process groups and the router talks to a pool leader directly:
  * ``send_obj`` / ``recv_obj``: length-prefixed byte messages (JSON: request batches, results);
  * ``send_tokens`` / ``recv_tokens``: int32 token-id tensors (failover hand-off of a prompt);
  * ``bcast_obj``: leader -> TP group fan-out of a work item;
  * ``ping``: 4 KiB ping-pong health probe, timed.
Calls made from a side thread run on a dedicated HIP stream (``side_stream``) so transfers
never queue behind the local engine's kernels on the default stream.
"""
from __future__ import annotations

import json
import time
from typing import Any, Optional

import torch
import torch.distributed as dist


def _dev(group) -> torch.device:
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def send_bytes(data: bytes, dst: int, group=None, tag: int = 0) -> None:
    dev = _dev(group)
    hdr = torch.tensor([len(data)], dtype=torch.int64, device=dev)
    dist.send(hdr, dst, group=group, tag=tag)
    if data:
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        dist.send(buf, dst, group=group, tag=tag)


def recv_bytes(src: int, group=None, tag: int = 0) -> bytes:
    dev = _dev(group)
    hdr = torch.empty(1, dtype=torch.int64, device=dev)
    dist.recv(hdr, src, group=group, tag=tag)
    n = int(hdr.item())
    if n == 0:
        return b""
    buf = torch.empty(n, dtype=torch.uint8, device=dev)
    dist.recv(buf, src, group=group, tag=tag)
    return bytes(buf.cpu().numpy().tobytes())


def send_obj(obj: Any, dst: int, group=None, tag: int = 0) -> None:
    send_bytes(json.dumps(obj).encode("utf-8"), dst, group, tag)


def recv_obj(src: int, group=None, tag: int = 0) -> Any:
    return json.loads(recv_bytes(src, group, tag).decode("utf-8"))


def bcast_obj(obj: Any, src: int, group=None) -> Any:
    """Broadcast a JSON-able object from global rank ``src`` to every member of ``group``."""
    dev = _dev(group)
    me = dist.get_rank()
    if me == src:
        data = json.dumps(obj).encode("utf-8")
        hdr = torch.tensor([len(data)], dtype=torch.int64, device=dev)
    else:
        hdr = torch.empty(1, dtype=torch.int64, device=dev)
    dist.broadcast(hdr, src, group=group)
    n = int(hdr.item())
    buf = (torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev) if me == src
           else torch.empty(n, dtype=torch.uint8, device=dev))
    dist.broadcast(buf, src, group=group)
    return obj if me == src else json.loads(bytes(buf.cpu().numpy().tobytes()).decode("utf-8"))


def send_tokens(ids, dst: int, group=None) -> None:
    dev = _dev(group)
    t = torch.as_tensor(ids, dtype=torch.int32).to(dev)
    dist.send(torch.tensor([t.numel()], dtype=torch.int64, device=dev), dst, group=group)
    dist.send(t, dst, group=group)


def recv_tokens(src: int, group=None) -> torch.Tensor:
    dev = _dev(group)
    hdr = torch.empty(1, dtype=torch.int64, device=dev)
    dist.recv(hdr, src, group=group)
    t = torch.empty(int(hdr.item()), dtype=torch.int32, device=dev)
    dist.recv(t, src, group=group)
    return t


def ping(peer: int, group=None, nbytes: int = 4096, initiator: bool = True) -> float:
    """4 KiB ping-pong; returns the round-trip time in microseconds on the initiator."""
    dev = _dev(group)
    buf = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
    t0 = time.perf_counter()
    if initiator:
        dist.send(buf, peer, group=group)
        dist.recv(buf, peer, group=group)
    else:
        dist.recv(buf, peer, group=group)
        dist.send(buf, peer, group=group)
    if dev.type == "cuda":
        torch.cuda.current_stream().synchronize()
    return (time.perf_counter() - t0) * 1e6


_side = {}


def side_stream(device: Optional[torch.device] = None):
    """A per-device side stream for pool-to-pool transfers (None on CPU)."""
    if not torch.cuda.is_available():
        return None
    d = torch.cuda.current_device() if device is None else torch.device(device).index
    if d not in _side:
        _side[d] = torch.cuda.Stream(device=d)
    return _side[d]
