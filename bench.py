#!/usr/bin/env python3
"""Flagship benchmark: routed end-to-end serving on MI355X (BASELINE.json metric).

Reference workload (src/tests/routing_chatbot_tester.py:405-486): each query set is replayed as
ONE growing conversation; every turn is routed (token / heuristic / semantic / hybrid / perf) to
the small or large tier and answered there; latency and response tokens are recorded per turn.

This bench runs BASELINE config 2 per GPU — TinyLlama-1.1B architecture (random-init bf16
weights, fixed seed: no checkpoints in this environment) serving BOTH tiers from one engine,
hybrid router with the semantic routing cache on (HBM-resident cache table, GPU MiniLM-L6
encoder).  Each GPU serves ``--convs`` concurrent conversations (the three reference query sets,
round-robin; every conversation gets a unique session tag so no two share KV prefixes or
responses).  One *step* = one turn of every conversation: route all, then the engine serves the
small-tier and large-tier groups as one continuous batch (paged KV, prefix cache across turns,
hipGraph decode).  The response cache is OFF (its context-free key would replay other
conversations' answers — skipped work), small tier greedy, large tier Ollama-default sampling.

Weak scaling: N ranks = N independent replicas (one process per GPU, RCCL for the
cross-rank reductions).  ``value`` = total generated tokens over all ranks / max rank time.

Output (rank 0, one JSON line): see the driver contract; extra keys: p50/p90 e2e latency per
routed turn, per-tier token split, routing mix, prefix-cache hit rate.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

BASELINE_TOK_S = 10.57        # best published routed throughput (Jetson Nano+Orin)
BASELINE_S_PER_QUERY = 39.6   # best published mean routed e2e latency per query


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="tinyllama-1.1b")
    ap.add_argument("--convs", type=int, default=64, help="concurrent conversations per GPU")
    ap.add_argument("--strategy", default="hybrid")
    ap.add_argument("--threshold", type=int, default=1000)
    ap.add_argument("--small-new", type=int, default=128)
    ap.add_argument("--large-new", type=int, default=384)
    ap.add_argument("--kv-gb", type=float, default=48.0)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--cpu", action="store_true", help="CPU plumbing run (tiny model)")
    return ap.parse_args()


def main() -> int:
    a = parse()
    import torch
    import torch.distributed as dist
    from distributed_llm_amd.bench.query_sets import normalize_query_set, query_sets
    from distributed_llm_amd.config import LARGE, PRODUCTION_CFG, SMALL
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    from distributed_llm_amd.orchestrator import Router
    from distributed_llm_amd.pools.base import EnginePool

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    on_gpu = torch.cuda.is_available() and not a.cpu
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if on_gpu:
            torch.cuda.set_device(local)
        dist.init_process_group("nccl" if on_gpu else "gloo")
    dev = f"cuda:{local}" if on_gpu else "cpu"
    model = a.model if on_gpu else "tiny-llama-test"
    if not on_gpu:
        os.environ.setdefault("DLLM_EMBEDDER", "hash")

    engine = LLMEngine(model, device=dev, kv_cache_gb=a.kv_gb if on_gpu else 0.2,
                       max_num_seqs=max(16, a.convs), use_graphs=not a.no_graphs, seed=0)
    pools = {SMALL: EnginePool(SMALL, engine, max_new_tokens=a.small_new, temperature=0.0),
             LARGE: EnginePool(LARGE, engine, max_new_tokens=a.large_new, temperature=0.8, top_k=40, top_p=0.9)}
    cfg = dict(PRODUCTION_CFG, token_threshold=a.threshold, enable_response_cache=False,
               cache_index_device=dev if on_gpu else None, cache_max_size=1 << 20)
    router = Router(strategy=a.strategy, config=cfg, threshold_fallback=a.threshold, benchmark_mode=False,
                    pools=pools)
    if on_gpu:
        engine.capture_all(max_bs=engine._bucket(a.convs))

    sets = [normalize_query_set(query_sets[k]) for k in ("general_knowledge", "technical_coding", "personal_health")]
    sessions = [0]

    def new_conv(i):
        sessions[0] += 1
        return {"set": sets[i % 3], "turn": 0, "hist": [], "tag": f"[session r{rank}-{sessions[0]}] "}

    convs = [new_conv(i) for i in range(a.convs)]
    records = []

    def step(record: bool):
        hs = []
        for c in convs:
            q = c["set"][c["turn"]].text
            if c["turn"] == 0:
                q = c["tag"] + q
            c["hist"].append({"role": "user", "content": q})
            hs.append(c["hist"])
        res = router.route_batch(hs)
        for i, (c, (payload, ntok, device)) in enumerate(zip(convs, res)):
            c["hist"].append({"role": "assistant", "content": payload["response"]})
            if record:
                raw = payload.get("raw") or {}
                records.append({"lat": float(raw.get("latency_ms", 0.0)), "tok": int(ntok), "dev": device,
                                "ovh": float(payload.get("routing_overhead_ms", 0.0)),
                                "ttft": float((raw.get("timing") or {}).get("ttft_ms", 0.0))})
            c["turn"] += 1
            if c["turn"] >= len(c["set"]):
                convs[i] = new_conv(i)

    def sync():
        if on_gpu:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    for _ in range(a.warmup):
        step(False)
    st0 = dict(engine.bm.stats())
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    sync()
    elapsed = time.perf_counter() - t0
    st1 = dict(engine.bm.stats())

    tokens = sum(r["tok"] for r in records)
    lats = sorted(r["lat"] for r in records)
    if world > 1:
        t = torch.tensor([float(tokens), elapsed], dtype=torch.float64, device=dev)
        tot = t.clone()
        dist.all_reduce(tot[:1], op=dist.ReduceOp.SUM)
        mx = t.clone()
        dist.all_reduce(mx[1:], op=dist.ReduceOp.MAX)
        tokens_all, elapsed_max = float(tot[0]), float(mx[1])
        lat_t = torch.tensor(lats, dtype=torch.float64)
        gathered = [None] * world
        dist.all_gather_object(gathered, lats)
        lats = sorted(x for g in gathered for x in g)
    else:
        tokens_all, elapsed_max = float(tokens), elapsed
    value = tokens_all / elapsed_max
    pct = lambda p: lats[min(len(lats) - 1, int(p * len(lats)))] if lats else 0.0
    n_small = sum(1 for r in records if r["dev"] == SMALL)
    hit = (st1["prefix_hit_tokens"] - st0["prefix_hit_tokens"]) / max(1, st1["prompt_tokens"] - st0["prompt_tokens"])
    if rank == 0:
        out = {
            "metric": "routed_tokens_per_sec",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed_max * 1000.0 / a.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_TOK_S, 2),
            "dtype": "bf16",
            "data": "synthetic: reference query sets replayed as growing conversations; random-init weights",
            "config": {"model": f"{model} (small+large tiers on one engine per GPU)" if on_gpu else model,
                       "global_batch": a.convs * world, "seq_len": "growing conversation (<=16384)",
                       "parallelism": f"dp{world}", "strategy": a.strategy, "semantic_cache": True,
                       "response_cache": False, "small_max_new": a.small_new, "large_max_new": a.large_new},
            "p50_latency_ms": round(statistics.median(lats), 1) if lats else None,
            "p90_latency_ms": round(pct(0.9), 1),
            "p50_latency_vs_baseline_mean_s_per_query": round(BASELINE_S_PER_QUERY * 1000.0 / max(1e-9, statistics.median(lats)), 1) if lats else None,
            "requests": len(lats),
            "small_tier_share": round(n_small / max(1, len(records)), 3),
            "routing_overhead_ms_mean": round(statistics.mean(r["ovh"] for r in records), 3) if records else None,
            "ttft_ms_p50": round(statistics.median(r["ttft"] for r in records), 1) if records else None,
            "prefix_cache_hit_rate": round(hit, 3),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
