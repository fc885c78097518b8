"""Pools that live on other ranks of the node, and data-parallel replica sets.

* ``RemotePool``  — the router-side client of a pool whose leader is another rank: request batches
  and results travel as point-to-point messages (parallel.p2p: RCCL send/recv over xGMI on a side
  HIP stream), replacing the reference's HTTP-over-SSH hop (src/models/nano.py:23-35).
* ``serve_pool``  — the pool-side loop: the leader receives work from the router and fans it out
  to its tensor-parallel group (every TP rank runs the same ``generate`` in lockstep; RCCL
  all-reduces inside the model), then returns the results.
* ``ReplicatedPool`` — several replicas of one tier (data parallel); a batch is split across
  replicas by outstanding load (least-loaded dispatch), replicas run concurrently.
"""
from __future__ import annotations

import itertools
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Dict, List, Optional, Sequence

from ..parallel import p2p
from .base import Coalescer, EnginePool, NullServerManager, PoolClient, format_prompt


class RemoteServerManager(NullServerManager):
    def __init__(self, pool: "RemotePool"):
        super().__init__()
        self.pool = pool

    def is_server_running(self) -> bool:
        return self.pool.alive


class RemotePool(PoolClient):
    def __init__(self, name: str, leader: int, group, max_new_tokens: int = 256, temperature: float = 0.0,
                 top_k: int = 0, top_p: float = 1.0, generation_prompt: str = EnginePool.GENERATION_PROMPT):
        super().__init__()
        self.name = name
        self.leader = leader
        self.group = group
        self.params = {"max_new_tokens": max_new_tokens, "temperature": temperature, "top_k": top_k, "top_p": top_p}
        self.generation_prompt = generation_prompt
        self.alive = True
        self.server_manager = RemoteServerManager(self)
        self._lock = threading.Lock()  # one outstanding exchange per pair group
        self._ids = itertools.count()
        self.last_rtt_us: Optional[float] = None
        self._coalesce = Coalescer(self._generate_items)  # concurrent callers -> one exchange

    def prompt_for(self, history: Any) -> str:
        return format_prompt(history) + self.generation_prompt

    def _exchange(self, msg: Dict[str, Any]) -> Dict[str, Any]:
        import torch
        st = p2p.side_stream()
        with self._lock:
            if st is not None:
                with torch.cuda.stream(st):
                    p2p.send_obj(msg, self.leader, self.group)
                    return p2p.recv_obj(self.leader, self.group)
            p2p.send_obj(msg, self.leader, self.group)
            return p2p.recv_obj(self.leader, self.group)

    def process(self, history: Any) -> Dict[str, Any]:
        return self.process_batch([history])[0]

    def process_batch(self, histories: Sequence[Any], overrides: Optional[Dict[str, Any]] = None):
        if not self.alive:
            return [{"error": f"pool {self.name} unavailable"}] * len(histories)
        params = dict(self.params, **(overrides or {}))
        return self._coalesce.submit([(self.prompt_for(h), params) for h in histories])

    def _generate_items(self, items: List[tuple]) -> List[Dict[str, Any]]:
        plist = [p for _, p in items]
        msg = {"op": "generate", "id": next(self._ids), "prompts": [q for q, _ in items]}
        if all(p == plist[0] for p in plist):
            msg["params"] = plist[0]
        else:
            msg["params_list"] = plist
        try:
            rep = self._exchange(msg)
        except Exception as e:  # transport failure -> error payloads (router fails over)
            self.alive = False
            return [{"error": f"pool {self.name} transport failed: {e}"}] * len(items)
        res = rep.get("results")
        if not res or len(res) != len(items):
            return [{"error": rep.get("error", "empty reply")}] * len(items)
        return res

    def probe(self) -> Dict[str, Any]:
        """Health probe: round trip + the pool's engine statistics."""
        t0 = time.perf_counter()
        try:
            rep = self._exchange({"op": "ping"})
        except Exception as e:
            self.alive = False
            return {"ok": False, "error": str(e)}
        self.last_rtt_us = (time.perf_counter() - t0) * 1e6
        return {"ok": True, "rtt_us": self.last_rtt_us, **rep.get("stats", {})}

    def health(self) -> Dict[str, Any]:
        return self.probe()

    def stop(self) -> None:
        if self.alive:
            with self._lock:
                p2p.send_obj({"op": "stop"}, self.leader, self.group)
            self.alive = False

    def sync(self) -> None:
        with self._lock:
            p2p.send_obj({"op": "sync"}, self.leader, self.group)


def serve_pool(engine, router_rank: int, leader: int, pair_group, tp_group=None, on_sync=None) -> None:
    """Pool-side loop (every rank of the pool calls it).  Returns on {"op": "stop"}."""
    import torch.distributed as dist
    from ..engine.sampling import SamplingParams
    me = dist.get_rank()
    while True:
        if me == leader:
            msg = p2p.recv_obj(router_rank, pair_group)
            if tp_group is not None:
                p2p.bcast_obj(msg, leader, tp_group)
        else:
            msg = p2p.bcast_obj(None, leader, tp_group)
        op = msg.get("op")
        if op == "stop":
            return
        if op == "sync":
            if on_sync is not None:
                on_sync()
            continue
        if op == "ping":
            if me == leader:
                p2p.send_obj({"op": "pong", "stats": {k: v for k, v in engine.stats().items()
                                                      if isinstance(v, (int, float, str))}}, router_rank, pair_group)
            continue
        if op == "generate":
            try:
                if "params_list" in msg:
                    sp = [SamplingParams(**p) for p in msg["params_list"]]
                else:
                    sp = SamplingParams(**msg["params"])
                outs = engine.generate(msg["prompts"], sp)
                res = EnginePool.to_payloads(outs)
                rep = {"id": msg["id"], "results": res}
            except Exception as e:  # report, never kill the pool loop
                rep = {"id": msg["id"], "error": f"engine failed: {e}"}
            if me == leader:
                p2p.send_obj(rep, router_rank, pair_group)


class ReplicatedPool(PoolClient):
    """Data-parallel replicas of one tier with least-loaded dispatch."""

    def __init__(self, name: str, replicas: List[PoolClient]):
        super().__init__()
        if not replicas:
            raise ValueError("need at least one replica")
        self.name = name
        self.replicas = replicas
        self.inflight = [0] * len(replicas)
        self._lock = threading.Lock()
        self._ex = ThreadPoolExecutor(max_workers=len(replicas))

    def _pick(self) -> int:
        with self._lock:
            i = min(range(len(self.replicas)), key=lambda k: self.inflight[k])
            self.inflight[i] += 1
            return i

    def process(self, history: Any) -> Dict[str, Any]:
        i = self._pick()
        try:
            return self.replicas[i].process(history)
        finally:
            with self._lock:
                self.inflight[i] -= 1

    def process_batch(self, histories: Sequence[Any]) -> List[Dict[str, Any]]:
        n = len(self.replicas)
        if n == 1 or len(histories) <= 1:
            return self.replicas[0].process_batch(histories) if n == 1 else [self.process(h) for h in histories]
        with self._lock:  # assign round-robin starting from the least-loaded replica
            order = sorted(range(n), key=lambda k: self.inflight[k])
            shards: Dict[int, List[int]] = {k: [] for k in range(n)}
            for j in range(len(histories)):
                shards[order[j % n]].append(j)
            for k, idx in shards.items():
                self.inflight[k] += len(idx)
        futs = {k: self._ex.submit(self.replicas[k].process_batch, [histories[j] for j in idx])
                for k, idx in shards.items() if idx}
        out: List[Any] = [None] * len(histories)
        for k, f in futs.items():
            try:
                res = f.result()
            finally:
                with self._lock:
                    self.inflight[k] -= len(shards[k])
            for j, r in zip(shards[k], res):
                out[j] = r
        return out

    def health(self) -> Dict[str, Any]:
        return {"ok": any(r.health().get("ok") for r in self.replicas), "replicas": len(self.replicas)}
