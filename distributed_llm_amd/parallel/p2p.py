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
On an RCCL pair group every data-plane transfer runs on a side HIP stream of its own (``side_stream``):
ProcessGroupNCCL orders a send/recv after the work queued on the CALLER's current stream, so on
the compute stream a failover hand-off or a probe would wait behind the decode graphs in flight;
on the side stream it waits only for its own staging copy.
Every data-plane wait can be bounded (``timeout_s``: isend / irecv + ``Work.wait(timeout)``); a
transfer past its deadline raises ``DataPlaneTimeout`` and the caller retires that pair group.
The data plane defaults to gloo (parallel.cluster): token ids and pings are tiny, and on gloo a
dead peer is a timeout exception in the calling thread rather than an RCCL watchdog abort of the
whole router process.
"""
from __future__ import annotations

import contextlib
import json
import threading
import time
from typing import Any, Dict, Iterator, Optional

import torch
import torch.distributed as dist


def _dev(group) -> torch.device:
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


_SIDE: Dict[int, "torch.cuda.Stream"] = {}
_SIDE_LOCK = threading.Lock()


def side_stream(dev: torch.device) -> Optional["torch.cuda.Stream"]:
    """The data plane's side stream on ``dev`` (one per device, created on first use); None on CPU."""
    if dev.type != "cuda":
        return None
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    with _SIDE_LOCK:
        s = _SIDE.get(idx)
        if s is None:
            s = _SIDE[idx] = torch.cuda.Stream(device=idx)
        return s


@contextlib.contextmanager
def on_side(dev: torch.device) -> Iterator[None]:
    """Run the enclosed transfer on the side stream and wait for it before leaving, so whatever the
    caller does next with the result (host copies, another stream) sees completed data."""
    s = side_stream(dev)
    if s is None:
        yield
        return
    with torch.cuda.stream(s):
        yield
    s.synchronize()


def send_bytes(data: bytes, dst: int, group=None, tag: int = 0, timeout_s: Optional[float] = None) -> None:
    """``timeout_s``: bound each transfer's wait (a send to a peer that died mid-conversation can
    block in gloo instead of raising); raises :class:`DataPlaneTimeout` when it passes."""
    dev = _dev(group)
    with on_side(dev):
        hdr = torch.tensor([len(data)], dtype=torch.int64, device=dev)
        _wait(dist.isend(hdr, dst, group=group, tag=tag), timeout_s, "send header")
        if data:
            buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
            _wait(dist.isend(buf, dst, group=group, tag=tag), timeout_s, "send payload")


def recv_bytes(src: int, group=None, tag: int = 0) -> bytes:
    dev = _dev(group)
    with on_side(dev):
        hdr = torch.empty(1, dtype=torch.int64, device=dev)
        dist.recv(hdr, src, group=group, tag=tag)
        n = int(hdr.item())
        if n == 0:
            return b""
        buf = torch.empty(n, dtype=torch.uint8, device=dev)
        dist.recv(buf, src, group=group, tag=tag)
        return bytes(buf.cpu().numpy().tobytes())


def send_obj(obj: Any, dst: int, group=None, tag: int = 0, timeout_s: Optional[float] = None) -> None:
    send_bytes(json.dumps(obj).encode("utf-8"), dst, group, tag, timeout_s)


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


class DataPlaneTimeout(RuntimeError):
    """A data-plane transfer did not complete within its deadline.  The pair group may still hold
    a posted receive, so callers stop using it (RemotePool falls back to the control plane)."""


def _wait(work, timeout_s: Optional[float], what: str) -> None:
    if timeout_s is None:
        work.wait()
        return
    from datetime import timedelta
    try:
        done = work.wait(timeout=timedelta(seconds=float(timeout_s)))
    except RuntimeError as e:   # gloo raises on its deadline
        raise DataPlaneTimeout(f"{what} timed out after {timeout_s}s: {e}") from e
    if done is False:
        raise DataPlaneTimeout(f"{what} timed out after {timeout_s}s")


def _send(t: torch.Tensor, dst: int, group, timeout_s: Optional[float], what: str) -> None:
    _wait(dist.isend(t, dst, group=group), timeout_s, what)


def _recv(t: torch.Tensor, src: int, group, timeout_s: Optional[float], what: str) -> None:
    _wait(dist.irecv(t, src, group=group), timeout_s, what)


def send_tokens(ids, dst: int, group=None, timeout_s: Optional[float] = None) -> None:
    """Ship int32 token ids (length header + payload); every wait is bounded by ``timeout_s``."""
    dev = _dev(group)
    with on_side(dev):
        t = torch.as_tensor(ids, dtype=torch.int32).to(dev)
        _send(torch.tensor([t.numel()], dtype=torch.int64, device=dev), dst, group, timeout_s, "token header send")
        if t.numel():
            _send(t, dst, group, timeout_s, "token send")


def recv_tokens(src: int, group=None, timeout_s: Optional[float] = None) -> torch.Tensor:
    dev = _dev(group)
    with on_side(dev):   # returns after the side stream drained: the ids are complete
        hdr = torch.empty(1, dtype=torch.int64, device=dev)
        _recv(hdr, src, group, timeout_s, "token header receive")
        t = torch.empty(int(hdr.item()), dtype=torch.int32, device=dev)
        if t.numel():
            _recv(t, src, group, timeout_s, "token receive")
    return t


def ping(peer: int, group=None, nbytes: int = 4096, initiator: bool = True,
         timeout_s: Optional[float] = None) -> float:
    """4 KiB ping-pong; returns the round-trip time in microseconds on the initiator."""
    dev = _dev(group)
    with on_side(dev):   # the round trip includes draining the side stream
        buf = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        t0 = time.perf_counter()
        if initiator:
            _send(buf, peer, group, timeout_s, "ping send")
            _recv(buf, peer, group, timeout_s, "ping receive")
        else:
            _recv(buf, peer, group, timeout_s, "ping receive")
            _send(buf, peer, group, timeout_s, "ping send")
    return (time.perf_counter() - t0) * 1e6
