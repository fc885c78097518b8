"""Build pool clients from a topology spec, and dispatch grouped requests.

Topology spec (``config["pools"]``)::

    {"nano": {"kind": "engine", "model": "tinyllama-1.1b", "device": "cuda:0",
              "max_new_tokens": 128, "temperature": 0.0, "share": "main"},
     "orin": {"kind": "engine", "model": "tinyllama-1.1b", "device": "cuda:0",
              "max_new_tokens": 384, "temperature": 0.8, "top_k": 40, "top_p": 0.9, "share": "main"}}

``share``: pools with the same share key and model use ONE engine (BASELINE config 2: one
model serving both tiers on one GPU).  ``kind`` may also be ``"http"`` (``url``: a pool
worker), ``"echo"``, or ``"supervised"``: a pool worker process this router starts and owns
(``port``, ``gpus``, ``tp``: one torchrun rank per GPU for tp > 1, ``worker_kind``), restarted
lazily by the next request after it died, as the reference's NanoModel restarts its device server
before a call (src/models/nano.py:19-21, server_manager.py:66-142) — the restartable form of a
large tensor-parallel pool (``data/topologies/supervised_pools_8gpu.json``).
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from typing import Any, Dict, List, Sequence, Tuple

from ..config import LARGE, SMALL, canonical_tier
from .base import EchoPool, EnginePool, HTTPPool, PoolClient, format_prompt


def build_pools(spec: Dict[str, Dict[str, Any]], supervisor=None) -> Dict[str, PoolClient]:
    """``supervisor``: the Supervisor that owns ``"supervised"`` workers (created on demand; the
    caller stops it with ``supervisor.stop_all()``, also reachable as ``pools[t].server_manager``)."""
    engines: Dict[Tuple[str, str], Any] = {}
    pools: Dict[str, PoolClient] = {}
    for name, s in spec.items():
        if name.startswith("_"):   # "_comment" and other annotations
            continue
        tier = canonical_tier(name)
        kind = s.get("kind", "engine")
        if kind == "echo":
            pools[tier] = EchoPool(tier, tokens_per_reply=int(s.get("max_new_tokens", 16)))
        elif kind == "http":
            pools[tier] = HTTPPool(tier, s["url"], timeout_s=float(s.get("timeout_s", 180.0)))
        elif kind == "supervised":
            from .supervisor import PoolSpec, Supervisor
            if supervisor is None:
                supervisor = Supervisor([], log_dir=s.get("log_dir", "gpurun_out/pools"),
                                        startup_timeout_s=float(s.get("startup_timeout_s", 300.0)))
            ps = PoolSpec(tier, int(s["port"]), gpus=[int(g) for g in s.get("gpus", [])],
                          kind=s.get("worker_kind", "engine"), model=s.get("model", "tinyllama-1.1b"),
                          max_new_tokens=int(s.get("max_new_tokens", 256)),
                          temperature=float(s.get("temperature", 0.0)), tp=int(s.get("tp", 1)),
                          extra_args=[str(x) for x in s.get("extra_args", [])])
            supervisor.specs[tier] = ps
            supervisor.restarts.setdefault(tier, 0)
            opts = {k: s[k] for k in ("top_k", "top_p") if k in s}
            pools[tier] = HTTPPool(tier, ps.url, timeout_s=float(s.get("timeout_s", 180.0)), supervisor=supervisor,
                                   options=opts)
            if s.get("start", True):
                supervisor.start(tier, wait=bool(s.get("wait", True)))
        elif kind == "engine":
            key = (s.get("share", tier), s["model"])
            eng = engines.get(key)
            if eng is None:
                from ..engine.llm_engine import LLMEngine
                eng = LLMEngine(s["model"], device=s.get("device", "cuda"), kv_cache_gb=s.get("kv_cache_gb"),
                                max_num_seqs=int(s.get("max_num_seqs", 256)),
                                max_model_len=s.get("max_model_len"), weights=s.get("weights"),
                                seed=int(s.get("seed", 0)), use_graphs=bool(s.get("graphs", True)))
                engines[key] = eng
            pools[tier] = EnginePool(tier, eng, max_new_tokens=int(s.get("max_new_tokens", 256)),
                                     temperature=float(s.get("temperature", 0.0)), top_k=int(s.get("top_k", 0)),
                                     top_p=float(s.get("top_p", 1.0)))
        else:
            raise ValueError(f"unknown pool kind {kind!r}")
    for t in (SMALL, LARGE):
        if t not in pools:
            raise ValueError(f"pool spec must define tier {t!r}")
    return pools


def dispatch_groups(pools: Dict[str, PoolClient], groups: Dict[str, List[Any]]) -> Dict[str, List[Dict[str, Any]]]:
    """Serve each tier's group; tiers that share one engine are served in ONE continuous batch."""
    out: Dict[str, List[Dict[str, Any]]] = {}
    eng_groups: Dict[int, List[str]] = {}
    for dev, hs in groups.items():
        p = pools[dev]
        if hs and isinstance(p, EnginePool):
            eng_groups.setdefault(id(p.engine), []).append(dev)
    done = set()
    for devs in eng_groups.values():
        if len(devs) < 2:
            continue
        engine = pools[devs[0]].engine
        prompts, params, owners = [], [], []
        for dev in devs:
            pp = pools[dev]._params()
            for h in groups[dev]:
                prompts.append(pools[dev].prompt_for(h))
                params.append(pp)
                owners.append(dev)
        res = EnginePool.to_payloads(engine.generate(prompts, params))
        for dev in devs:
            out[dev] = []
        for dev, r in zip(owners, res):
            out[dev].append(r)
        done.update(devs)
    rest = [dev for dev, hs in groups.items() if dev not in done and hs]
    if len(rest) == 1:
        out[rest[0]] = pools[rest[0]].process_batch(groups[rest[0]])
    elif rest:  # different pools (other GPUs / other ranks) serve their groups concurrently
        with ThreadPoolExecutor(max_workers=len(rest)) as ex:
            futs = {dev: ex.submit(pools[dev].process_batch, groups[dev]) for dev in rest}
            for dev, f in futs.items():
                out[dev] = f.result()
    return out
