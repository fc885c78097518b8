"""Node topology: small / large tier pools on GPU subsets (one process per GPU).

BASELINE.json configs 3-5: "Llama-3-1B (small pool, GPU0) + Llama-3-8B (large pool, GPU1)",
"8B small pool (2 GPUs) + 70B TP=4 large pool", "Mixtral TP=8 large + 1B small co-located".
The reference's equivalent is two models served side by side behind one router, each on its own
board behind an SSH tunnel (src/devices/nano_api.py:15-16, orin_api.py:17-18; dispatch at
src/router.py:152-171; lifecycle src/models/server_manager.py).

``Topology`` lists the replicas of each tier as rank lists (a replica with > 1 rank is one
tensor-parallel group).  A rank may host more than one replica (``colocated``: BASELINE config 5's
small pool shares the GPUs of the large pool's TP group; each replica is its own engine, sized by
its TierSpec's ``kv_cache_gb``: memory partitioning on the shared 288 GB).  ``Cluster`` (every
rank constructs it, in the same order) creates the process groups, loads this rank's engine(s),
and then either
  * rank 0 (router rank): ``router_pools()`` -> {tier: PoolClient} mixing its local engines,
    remote pools (``pools.remote.RemotePool``: tagged control messages on a gloo pair group, token
    ids on the data-plane pair group — gloo by default, RCCL with ``DLLM_DATA_PLANE=rccl``) and
    replica sets (``ReplicatedPool``); or
  * every other rank: ``serve()`` — one serving loop per replica it hosts (a remote pool leader's
    request loop, a TP member's scheduler mirror), until the router sends stop.
Default layouts (``default_topology``): 1 GPU — both tiers on one engine; 2 — small [0], large [1];
4 — small replicas [0], [1], large TP=2 [2, 3]; 8 — small replicas [0]..[3], large TP=4 [4..7];
colocated (config 5) — small replicas [0]..[N-1], large TP=N [0..N-1] on the same GPUs.
RCCL carries the TP groups' collectives only.
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


def model_name(model) -> str:
    """A TierSpec's model: a registry name, or a ``ModelConfig`` (e.g. layer-truncated rehearsals)."""
    return model if isinstance(model, str) else model.name


def model_config(model):
    from ..models.configs import get_model_config
    return get_model_config(model) if isinstance(model, str) else model


@dataclass
class TierSpec:
    model: Any = "tinyllama-1.1b"     # registry name or models.configs.ModelConfig
    max_new_tokens: int = 256
    temperature: float = 0.0
    top_k: int = 0
    top_p: float = 1.0
    kv_cache_gb: Optional[float] = None
    max_num_seqs: int = 256
    graphs: bool = True          # hipGraph decode (off: eager steps, e.g. gloo collectives)


@dataclass
class Topology:
    replicas: Dict[str, List[List[int]]] = field(default_factory=dict)

    def all_groups(self):
        for tier in (SMALL, LARGE):
            for ranks in self.replicas.get(tier, []):
                yield tier, ranks


def default_topology(world: int, large_tp: Optional[int] = None, colocated: bool = False) -> Topology:
    if colocated:
        # BASELINE config 5: the large pool's TP group(s) span the node and every GPU also hosts a
        # small-tier replica (two engines per process)
        tp = large_tp or world
        if world % tp:
            raise ValueError(f"large tp={tp} must divide {world}")
        return Topology({SMALL: [[r] for r in range(world)],
                         LARGE: [list(range(i, i + tp)) for i in range(0, world, tp)]})
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
                 shared_single: bool = True, request_timeout_s: float = 180.0):
        self.topo = topo
        self.specs = specs
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.device = device or ("cuda" if torch.cuda.is_available() else "cpu")
        self.request_timeout_s = request_timeout_s
        self.sync_times: List[float] = []
        self.degraded = False   # or a reason string: a rank of the node died
        # --- groups (collective: every rank creates every group in the same order)
        #   tp_groups:     RCCL (default backend) per TP replica: model all-reduces
        #   mirror_groups: gloo per TP replica: the leader's scheduler broadcast (engine mirror)
        #   pair_groups:   router <-> remote leader: data plane (token ids, pings); gloo unless
        #                  DLLM_DATA_PLANE=rccl (a dead peer is then an exception in the calling
        #                  thread, never an RCCL watchdog abort of the router process), so RCCL
        #                  carries only the TP collectives
        #   ctrl_groups:   router <-> remote leader, gloo: tagged control messages (pools.remote)
        self.tp_groups: Dict[tuple, Any] = {}
        self.mirror_groups: Dict[tuple, Any] = {}
        self.pair_groups: Dict[int, Any] = {}
        self.ctrl_groups: Dict[int, Any] = {}
        init = dist.is_initialized()
        for tier, ranks in topo.all_groups():
            key = tuple(ranks)
            if len(ranks) > 1 and key not in self.tp_groups and init:
                self.tp_groups[key] = dist.new_group(list(ranks))
                self.mirror_groups[key] = dist.new_group(list(ranks), backend="gloo")
        remote = [ranks for _, ranks in topo.all_groups() if ranks[0] != 0]
        leaders = sorted({ranks[0] for ranks in remote})
        if len(leaders) != len({tuple(r) for r in remote}):
            # one control / data pair group per remote leader: two remote replicas led by one rank
            # would share (and interleave on) it
            raise ValueError(f"a rank other than 0 leads two remote replicas: {remote}")
        import os
        data_backend = None if os.environ.get("DLLM_DATA_PLANE", "gloo") == "rccl" else "gloo"
        for ld in leaders:
            self.pair_groups[ld] = dist.new_group([0, ld], backend=data_backend) if init else None
            self.ctrl_groups[ld] = dist.new_group([0, ld], backend="gloo") if init else None
        # --- this rank's replica(s): one, or several when tiers share GPUs (co-located pools, or
        # both tiers on one engine at world 1); every rank builds them in all_groups() order, so
        # the TP groups' collective set-up (custom all-reduce handles) lines up across ranks
        self.my: List[tuple] = [(tier, ranks) for tier, ranks in topo.all_groups() if self.rank in ranks]
        self.engines: Dict[tuple, Any] = {}
        from ..engine.llm_engine import LLMEngine
        for tier, ranks in self.my:
            spec = specs[tier]
            key = (tuple(ranks), model_name(spec.model))
            if key in self.engines:
                continue
            par = ParallelContext(len(ranks), ranks.index(self.rank), self.tp_groups.get(tuple(ranks)),
                                  self.rank, self.world)
            if str(self.device).startswith("cuda"):
                par.enable_custom_all_reduce(self.device)  # collective over this TP group
            eng = LLMEngine(spec.model, device=self.device, par=par, kv_cache_gb=spec.kv_cache_gb,
                            max_num_seqs=spec.max_num_seqs, use_graphs=spec.graphs)
            if len(ranks) > 1:
                eng.enable_tp_mirror(self.mirror_groups[tuple(ranks)], ranks[0])
            self.engines[key] = eng

    # ------------------------------------------------------------------ router side
    def _engine_for(self, tier: str, ranks: List[int]):
        return self.engines[(tuple(ranks), model_name(self.specs[tier].model))]

    def router_pools(self, on_health=None, probe_interval_s: Optional[float] = None):
        """{tier: PoolClient} for the router on rank 0.  ``on_health(name, ok, rtt_us)`` receives
        every remote health probe (``probe_interval_s``: start periodic probes)."""
        from ..engine.tokenizer import get_tokenizer
        from ..models.configs import get_model_config
        from ..pools.base import EnginePool
        from ..pools.remote import RemotePool, ReplicatedPool
        assert self.rank == 0, "router pools live on rank 0"
        out = {}
        self.remotes: List[RemotePool] = []
        self.local_engines = []
        for tier in (SMALL, LARGE):
            spec = self.specs[tier]
            reps = []
            for ranks in self.topo.replicas[tier]:
                kw = dict(max_new_tokens=spec.max_new_tokens, temperature=spec.temperature, top_k=spec.top_k,
                          top_p=spec.top_p)
                if 0 in ranks:
                    eng = self._engine_for(tier, ranks)
                    if len(ranks) > 1:   # rank 0 leads a TP group: members follow its scheduler
                        eng.start()
                        self.local_engines.append(eng)
                    reps.append(EnginePool(tier, eng, **kw))
                else:
                    cfg = model_config(spec.model)
                    rp = RemotePool(tier, ranks[0], self.ctrl_groups[ranks[0]], self.pair_groups[ranks[0]],
                                    timeout_s=self.request_timeout_s, on_health=on_health,
                                    tokenizer=get_tokenizer(cfg.vocab, cfg.bos_id, cfg.eos_id), **kw)
                    if probe_interval_s:
                        rp.start_probes(probe_interval_s)
                    reps.append(rp)
                    self.remotes.append(rp)
            out[tier] = reps[0] if len(reps) == 1 else ReplicatedPool(tier, reps)
        return out

    def sync(self) -> None:
        """Barrier across the whole node (router + every pool rank)."""
        if self.world == 1:
            return
        for rp in getattr(self, "remotes", []):
            if rp.alive:
                rp.sync()
        for eng in getattr(self, "local_engines", []):
            eng.mirror_control({"sync": True})
        self._barrier()

    def _barrier(self) -> None:
        """Node-wide barrier.  A rank that died (a pool process lost mid-run) makes the barrier
        fail on every survivor: the node is then ``degraded`` and later barriers are skipped, so
        the survivors still finish (the bench reduces its results through the rendezvous store,
        which outlives any non-zero rank)."""
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if not self.degraded:
            try:
                dist.barrier()
            except Exception as e:  # noqa: BLE001 - a peer died (gloo: connection closed)
                self.degraded = f"node barrier failed: {e}"
        self.sync_times.append(time.perf_counter())

    def shutdown(self) -> None:
        if self.rank != 0:
            return
        for rp in getattr(self, "remotes", []):
            rp.stop()
        for eng in getattr(self, "local_engines", []):
            eng.stop()   # mirror leader: sends stop to its members

    # ------------------------------------------------------------------ pool side
    def serve(self) -> None:
        """Pool ranks: a remote leader serves the router's requests; TP members follow their
        leader's scheduler.  A rank hosting several replicas runs one loop per replica (threads of
        this process) and joins each node-wide sync ONCE, when all its loops have reached it.
        Returns when the router has stopped every pool this rank serves."""
        from ..pools.remote import PoolLeader
        assert self.rank != 0
        loops = []
        seen = set()
        for tier, ranks in self.my:
            eng = self._engine_for(tier, ranks)
            if id(eng) in seen:
                continue
            seen.add(id(eng))
            loops.append((eng, ranks))
        on_sync = self._barrier
        gate = threading.Barrier(len(loops), action=self._barrier) if len(loops) > 1 else None
        if gate is not None:
            def on_sync():
                try:
                    gate.wait()
                except threading.BrokenBarrierError:   # a co-located loop ended (its pool died)
                    self._barrier()

        def run(eng, ranks):
            if self.rank == ranks[0]:
                PoolLeader(eng, self.ctrl_groups[self.rank], self.pair_groups[self.rank], 0,
                           on_sync=on_sync).serve()
                return
            try:
                eng.follow(on_sync=on_sync)
            except Exception as e:  # noqa: BLE001 - the TP leader's process died: this pool is gone
                import logging
                self.degraded = f"TP leader rank {ranks[0]} lost: {e}"
                logging.getLogger(__name__).error("TP member of %s: %s", ranks, self.degraded)
                if gate is not None:
                    gate.abort()   # co-located loops on this rank must not wait for this one

        errors: List[BaseException] = []

        def guarded(eng, ranks):
            try:
                run(eng, ranks)
            except BaseException as e:  # noqa: BLE001 - re-raised on the serving thread
                errors.append(e)

        threads = [threading.Thread(target=guarded, args=lp, name=f"dllm-serve-{lp[1][0]}", daemon=True)
                   for lp in loops[1:]]
        for t in threads:
            t.start()
        run(*loops[0])
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
