"""Node topology: small / large tier pools on disjoint GPU subsets (one process per GPU).

BASELINE.json configs 3-5: "Llama-3-1B (small pool, GPU0) + Llama-3-8B (large pool, GPU1)",
"8B small pool (2 GPUs) + 70B TP=4 large pool", "Mixtral TP=8 large + 1B small co-located".
The reference's equivalent is two boards behind SSH tunnels (src/models/server_manager.py).

``Topology`` lists the replicas of each tier as rank lists (a replica with > 1 rank is one
tensor-parallel group).  ``Cluster`` (every rank constructs it, in the same order) creates the
process groups, loads this rank's engine, and then either
  * rank 0 (router rank): ``router_pools()`` -> {tier: PoolClient} mixing its local engine, remote
    pools (``pools.remote.RemotePool`` over RCCL P2P) and replica sets (``ReplicatedPool``); or
  * every other rank: ``serve()`` — the pool loop until the router sends stop.
Default layouts (``default_topology``): 1 GPU — both tiers on one engine; 2 — small [0], large [1];
4 — small replicas [0], [1], large TP=2 [2, 3]; 8 — small replicas [0]..[3], large TP=4 [4..7].
"""
from __future__ import annotations

import threading

import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import torch
import torch.distributed as dist

from ..config import LARGE, SMALL
from .comm import ParallelContext


@dataclass
class TierSpec:
    model: str = "tinyllama-1.1b"
    max_new_tokens: int = 256
    temperature: float = 0.0
    top_k: int = 0
    top_p: float = 1.0
    kv_cache_gb: Optional[float] = None
    max_num_seqs: int = 256


@dataclass
class Topology:
    replicas: Dict[str, List[List[int]]] = field(default_factory=dict)

    def all_groups(self):
        for tier in (SMALL, LARGE):
            for ranks in self.replicas.get(tier, []):
                yield tier, ranks


def default_topology(world: int, large_tp: Optional[int] = None) -> Topology:
    if world == 1:
        return Topology({SMALL: [[0]], LARGE: [[0]]})
    if world == 2:
        return Topology({SMALL: [[0]], LARGE: [[1]]})
    half = world // 2
    tp = large_tp or half
    if half % tp:
        raise ValueError(f"large tp={tp} must divide {half}")
    large = [list(range(half + i, half + i + tp)) for i in range(0, half, tp)]
    return Topology({SMALL: [[r] for r in range(half)], LARGE: large})


class Cluster:
    def __init__(self, topo: Topology, specs: Dict[str, TierSpec], device: Optional[str] = None,
                 shared_single: bool = True):
        self.topo = topo
        self.specs = specs
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.device = device or ("cuda" if torch.cuda.is_available() else "cpu")
        self.sync_times: List[float] = []
        # --- groups (collective: every rank creates every group in the same order)
        self.tp_groups: Dict[tuple, Any] = {}
        self.pair_groups: Dict[int, Any] = {}
        for tier, ranks in topo.all_groups():
            key = tuple(ranks)
            if len(ranks) > 1 and key not in self.tp_groups and dist.is_initialized():
                self.tp_groups[key] = dist.new_group(list(ranks))
        leaders = sorted({ranks[0] for _, ranks in topo.all_groups() if ranks[0] != 0})
        for ld in leaders:
            self.pair_groups[ld] = dist.new_group([0, ld]) if dist.is_initialized() else None
        # --- this rank's replica(s): a rank serves exactly one replica (both tiers only if shared)
        self.my: List[tuple] = [(tier, ranks) for tier, ranks in topo.all_groups() if self.rank in ranks]
        self.engines: Dict[tuple, Any] = {}
        from ..engine.llm_engine import LLMEngine
        for tier, ranks in self.my:
            spec = specs[tier]
            key = (tuple(ranks), spec.model)
            if key in self.engines:
                continue
            par = ParallelContext(len(ranks), ranks.index(self.rank), self.tp_groups.get(tuple(ranks)),
                                  self.rank, self.world)
            if str(self.device).startswith("cuda"):
                par.enable_custom_all_reduce(self.device)  # collective over this TP group
            self.engines[key] = LLMEngine(spec.model, device=self.device, par=par, kv_cache_gb=spec.kv_cache_gb,
                                          max_num_seqs=spec.max_num_seqs)

    # ------------------------------------------------------------------ router side
    def _engine_for(self, tier: str, ranks: List[int]):
        return self.engines[(tuple(ranks), self.specs[tier].model)]

    def router_pools(self):
        from ..pools.base import EnginePool
        from ..pools.remote import RemotePool, ReplicatedPool
        assert self.rank == 0, "router pools live on rank 0"
        out = {}
        self.remotes: List[RemotePool] = []
        for tier in (SMALL, LARGE):
            spec = self.specs[tier]
            reps = []
            for ranks in self.topo.replicas[tier]:
                kw = dict(max_new_tokens=spec.max_new_tokens, temperature=spec.temperature, top_k=spec.top_k,
                          top_p=spec.top_p)
                if 0 in ranks:
                    if len(ranks) > 1:
                        reps.append(_LeaderPool(tier, self._engine_for(tier, ranks), self.tp_groups[tuple(ranks)],
                                                **kw))
                    else:
                        reps.append(EnginePool(tier, self._engine_for(tier, ranks), **kw))
                else:
                    rp = RemotePool(tier, ranks[0], self.pair_groups[ranks[0]], **kw)
                    reps.append(rp)
                    self.remotes.append(rp)
            out[tier] = reps[0] if len(reps) == 1 else ReplicatedPool(tier, reps)
        return out

    def sync(self) -> None:
        """Barrier across the whole node (router + every pool rank)."""
        if self.world == 1:
            return
        for rp in getattr(self, "remotes", []):
            rp.sync()
        for tier, ranks in self.my:
            if len(ranks) > 1 and ranks[0] == 0:
                from . import p2p
                p2p.bcast_obj({"op": "sync"}, 0, self.tp_groups[tuple(ranks)])
                break
        self._barrier()

    def _barrier(self) -> None:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        dist.barrier()
        self.sync_times.append(time.perf_counter())

    def shutdown(self) -> None:
        if self.rank != 0:
            return
        for rp in getattr(self, "remotes", []):
            rp.stop()
        for tier, ranks in self.my:
            if len(ranks) > 1 and ranks[0] == 0:
                from . import p2p
                p2p.bcast_obj({"op": "stop"}, 0, self.tp_groups[tuple(ranks)])
                break

    # ------------------------------------------------------------------ pool side
    def serve(self) -> None:
        from ..pools.remote import serve_pool
        assert self.rank != 0
        tier, ranks = self.my[0]
        eng = self._engine_for(tier, ranks)
        leader = ranks[0]
        serve_pool(eng, 0, leader, self.pair_groups.get(leader), self.tp_groups.get(tuple(ranks)),
                   on_sync=self._barrier)


class _LeaderPool:
    """Rank 0 leads a TP group: fan the request out to the members, then run it locally."""

    def __new__(cls, tier, engine, tp_group, **kw):
        from ..pools.base import Coalescer, EnginePool

        class LeaderPool(EnginePool):
            """Concurrent callers are coalesced into ONE broadcast + generate, so the members see
            requests in exactly the leader's order and batch as the leader does."""

            def __init__(self, *a, **k):
                super().__init__(*a, **k)
                self._coalesce = Coalescer(self._run_items)

            def process_batch(self, histories, overrides=None):
                params = self._params(overrides)
                return self._coalesce.submit([(self.prompt_for(h), params) for h in histories])

            def _run_items(self, items):
                from . import p2p
                prompts = [q for q, _ in items]
                plist = [p for _, p in items]
                p2p.bcast_obj({"op": "generate", "id": 0, "prompts": prompts,
                               "params_list": [{"max_new_tokens": p.max_new_tokens, "temperature": p.temperature,
                                                "top_k": p.top_k, "top_p": p.top_p} for p in plist]}, 0, tp_group)
                return self.to_payloads(self.engine.generate(prompts, plist))

        return LeaderPool(tier, engine, **kw)
