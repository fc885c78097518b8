"""Routing benchmark harness — reference CSV schemas, MI355X pools.

Reference: ``src/tests/routing_chatbot_tester.py`` (CLI :610-633, experiment loop :322-603,
per-query schema :334-341, summary schema :323-332, accuracy :293-298, warm-up :284-290,
cache clearing :273-281, config building :261-270).

Same experiment semantics: thresholds are swept only for the ``token`` strategy, other strategies
run once at ``--fixed-threshold`` (default: last of ``--thresholds``); each experiment builds a
fresh Router, clears the routing cache, sends one warm-up turn, then replays the query set as ONE
growing conversation; per-query and summary rows use the reference column names and order.
Extra columns are appended AFTER the reference columns (``gpus, small_pool, large_pool,
ttft_ms, prefill_tokens, cached_tokens`` per query; ``gpus, p50_latency_ms, p90_latency_ms,
tokens_per_sec, mean_ttft_ms`` per summary row).  Differences by design: no SSH (pools are local),
energy from amdsmi GPU socket power sampled at 10 Hz (``bench.power``), rows are appended as each
experiment finishes (``--resume`` skips experiments already in the summary CSV), and CLI flags are
never overridden by hard-coded argv (quirk 6).
"""
from __future__ import annotations

import argparse
import csv
import os
import statistics
from dataclasses import dataclass
from datetime import datetime
from typing import Any, Dict, List, Optional, Sequence, Tuple

from ..config import BENCHMARK_CFG, LARGE, PRODUCTION_CFG, SMALL
from .power import PowerSampler
from .query_sets import QueryItem, normalize_query_set, query_sets

SUMMARY_HEADERS = [
    "query_set", "strategy", "cache_mode", "token_threshold",
    "routing_accuracy",
    "nano_total_latency_ms", "nano_total_energy_mJ", "nano_avg_power_mW", "nano_total_tokens",
    "nano_latency_per_token_ms", "nano_energy_per_token_mJ",
    "orin_total_latency_ms", "orin_total_energy_mJ", "orin_avg_power_mW", "orin_total_tokens",
    "orin_latency_per_token_ms", "orin_energy_per_token_mJ",
    "overall_total_latency_ms", "overall_total_energy_mJ", "overall_total_tokens",
    "overall_latency_per_token_ms", "overall_energy_per_token_mJ",
]
# extra columns appended after the reference's; tokens_per_sec counts like the reference (TokenCounter on
# the returned text), generated_tokens_per_sec counts the tokens the engine actually decoded
SUMMARY_EXTRA = ["gpus", "p50_latency_ms", "p90_latency_ms", "tokens_per_sec", "mean_ttft_ms",
                 "generated_tokens", "generated_tokens_per_sec"]

PER_QUERY_HEADERS = [
    "query_set", "strategy", "cache_mode", "token_threshold",
    "query_index", "query_text", "expected_device",
    "device_used", "cache_hit",
    "routing_method", "routing_confidence", "routing_reasoning", "routing_overhead_ms",
    "start_time", "end_time", "latency_ms", "response_tokens",
    "energy_mJ", "latency_per_token_ms", "energy_per_token_mJ",
]
PER_QUERY_EXTRA = ["gpus", "small_pool", "large_pool", "ttft_ms", "prefill_tokens", "cached_tokens",
                   "generated_tokens", "energy_method", "energy_gpus"]


@dataclass
class RunConfig:
    query_set_name: str
    thresholds: List[int]
    strategies: List[str]
    cache_modes: List[str]
    fixed_threshold_for_non_token: int
    output_csv: str
    output_per_query_csv: str
    resume: bool = False


def build_router_config(cache_enabled: bool, token_threshold: int, extra: Optional[Dict[str, Any]] = None):
    base = PRODUCTION_CFG if cache_enabled else BENCHMARK_CFG
    cfg = {**base, "token_threshold": token_threshold}
    if extra:
        cfg.update(extra)
    return cfg


def compute_accuracy(rows: Sequence[Dict[str, Any]]) -> Optional[float]:
    lab = [r for r in rows if r.get("expected_device") in (SMALL, LARGE)]
    if not lab:
        return None
    return sum(1 for r in lab if r.get("device_used") == r.get("expected_device")) / len(lab)


def _ensure_header(path: str, headers: List[str]) -> None:
    if os.path.exists(path) and os.path.getsize(path) > 0:
        return
    with open(path, "w", newline="") as f:
        csv.writer(f).writerow(headers)


def _append(path: str, headers: List[str], row: Dict[str, Any]) -> None:
    with open(path, "a", newline="") as f:
        csv.writer(f).writerow([row.get(h, "") for h in headers])


def _done_keys(path: str) -> set:
    if not os.path.exists(path):
        return set()
    with open(path, newline="") as f:
        return {(r["query_set"], r["strategy"], r["cache_mode"], int(r["token_threshold"]))
                for r in csv.DictReader(f)}


def summarize(rows: List[Dict[str, Any]], query_set: str, strategy: str, cache_mode: str, thr: int,
              gpus: int) -> Dict[str, Any]:
    acc = compute_accuracy(rows)

    def agg(dev):
        sel = [r for r in rows if r.get("device_used") == dev]
        return (sum(int(r["latency_ms"] or 0) for r in sel), sum(float(r["energy_mJ"] or 0.0) for r in sel),
                sum(int(r["response_tokens"] or 0) for r in sel))

    out: Dict[str, Any] = {"query_set": query_set, "strategy": strategy, "cache_mode": cache_mode,
                           "token_threshold": thr, "routing_accuracy": "" if acc is None else round(acc, 4)}
    tot_l = tot_e = tot_t = 0
    for dev in (SMALL, LARGE):
        lat, e, t = agg(dev)
        tot_l, tot_e, tot_t = tot_l + lat, tot_e + e, tot_t + t
        out.update({
            f"{dev}_total_latency_ms": lat, f"{dev}_total_energy_mJ": round(e, 3),
            f"{dev}_avg_power_mW": round(e / (lat / 1000.0), 6) if lat > 0 else 0.0,
            f"{dev}_total_tokens": t,
            f"{dev}_latency_per_token_ms": round(lat / t, 6) if t > 0 else "",
            f"{dev}_energy_per_token_mJ": round(e / t, 6) if t > 0 else ""})
    out.update({"overall_total_latency_ms": tot_l, "overall_total_energy_mJ": round(tot_e, 3),
                "overall_total_tokens": tot_t,
                "overall_latency_per_token_ms": round(tot_l / tot_t, 6) if tot_t > 0 else "",
                "overall_energy_per_token_mJ": round(tot_e / tot_t, 6) if tot_t > 0 else ""})
    lats = sorted(int(r["latency_ms"] or 0) for r in rows if r.get("device_used") in (SMALL, LARGE))
    ttfts = [float(r["ttft_ms"]) for r in rows if r.get("ttft_ms") not in ("", None)]
    out.update({"gpus": gpus,
                "p50_latency_ms": statistics.median(lats) if lats else "",
                "p90_latency_ms": lats[min(len(lats) - 1, int(0.9 * len(lats)))] if lats else "",
                "tokens_per_sec": round(tot_t / (tot_l / 1000.0), 3) if tot_l > 0 else "",
                "mean_ttft_ms": round(statistics.mean(ttfts), 3) if ttfts else ""})
    gen = [int(r["generated_tokens"]) for r in rows if r.get("generated_tokens") not in ("", None)]
    out.update({"generated_tokens": sum(gen) if gen else "",
                "generated_tokens_per_sec": round(sum(gen) / (tot_l / 1000.0), 3) if gen and tot_l > 0 else ""})
    return out


def run_experiment(items: List[QueryItem], cfg: RunConfig, pools, tier_gpus: Dict[str, List[int]],
                   sampler: Optional[PowerSampler] = None, pool_names: Optional[Dict[str, str]] = None,
                   router_extra: Optional[Dict[str, Any]] = None, log=print) -> List[Dict[str, Any]]:
    from ..orchestrator import Router
    hdr_s, hdr_q = SUMMARY_HEADERS + SUMMARY_EXTRA, PER_QUERY_HEADERS + PER_QUERY_EXTRA
    _ensure_header(cfg.output_csv, hdr_s)
    _ensure_header(cfg.output_per_query_csv, hdr_q)
    done = _done_keys(cfg.output_csv) if cfg.resume else set()
    gpus = len({g for v in tier_gpus.values() for g in v}) or 0
    pool_names = pool_names or {}
    summaries = []
    for strategy in cfg.strategies:
        for cache_mode in cfg.cache_modes:
            cache_on = cache_mode.lower() == "on"
            thrs = cfg.thresholds if strategy == "token" else [cfg.fixed_threshold_for_non_token]
            for thr in thrs:
                if (cfg.query_set_name, strategy, cache_mode, int(thr)) in done:
                    log(f"[resume] skip {strategy}/{cache_mode}/{thr}")
                    continue
                try:
                    router = Router(strategy=strategy, config=build_router_config(cache_on, thr, router_extra),
                                    threshold_fallback=thr, benchmark_mode=not cache_on, pools=pools)
                except Exception as e:
                    log(f"[skip] strategy={strategy} cache={cache_mode} thr={thr} -> {e}")
                    continue
                log(f"[run] strategy={strategy} cache={cache_mode} benchmark_mode={not cache_on} threshold={thr}")
                for p in (router.nano, router.orin):
                    try:
                        p.server_manager.start_server()
                    except Exception:
                        pass
                router.query_router.clear_cache()
                try:
                    router.route_query([{"role": "user", "content": "Reply with exactly: OK"}])
                except Exception:
                    pass
                history: List[Dict[str, str]] = []
                rows: List[Dict[str, Any]] = []
                for i, it in enumerate(items):
                    history.append({"role": "user", "content": it.text})
                    m0 = sampler.mark() if sampler is not None else None
                    t0 = datetime.now()
                    row = {"query_set": cfg.query_set_name, "strategy": strategy, "cache_mode": cache_mode,
                           "token_threshold": thr, "query_index": i, "query_text": it.text,
                           "expected_device": it.expected_device, "gpus": gpus,
                           "small_pool": pool_names.get(SMALL, ""), "large_pool": pool_names.get(LARGE, "")}
                    try:
                        payload, ntok, dev = router.route_query(history)
                    except Exception as e:
                        t1 = datetime.now()
                        row["_marks"] = (m0, sampler.mark() if sampler is not None else None)
                        row.update({"device_used": "error", "start_time": t0, "end_time": t1,
                                    "latency_ms": int((t1 - t0).total_seconds() * 1000), "response_tokens": 0,
                                    "energy_mJ": 0.0})
                        rows.append(row)
                        log(f"[err] strategy={strategy} i={i}: {e}")
                        continue
                    t1 = datetime.now()
                    row["_marks"] = (m0, sampler.mark() if sampler is not None else None)
                    text = str(payload.get("response", "")) if isinstance(payload, dict) else str(payload)
                    history.append({"role": "assistant", "content": text})
                    timing = (payload.get("timing") or {}) if isinstance(payload, dict) else {}
                    row.update({
                        "device_used": dev, "cache_hit": payload.get("cache_hit", ""),
                        "routing_method": payload.get("routing_method", ""),
                        "routing_confidence": payload.get("routing_confidence", ""),
                        "routing_reasoning": payload.get("routing_reasoning", ""),
                        "routing_overhead_ms": payload.get("routing_overhead_ms", ""),
                        "start_time": t0, "end_time": t1, "latency_ms": int((t1 - t0).total_seconds() * 1000),
                        "response_tokens": int(ntok or 0), "ttft_ms": timing.get("ttft_ms", ""),
                        "prefill_tokens": timing.get("prefill_tokens", ""),
                        "cached_tokens": timing.get("cached_tokens", ""),
                        "generated_tokens": timing.get("generated_tokens", "")
                        if timing.get("generated_tokens") is not None else ""})
                    rows.append(row)
                for r in rows:
                    dev = r.get("device_used")
                    marks = r.pop("_marks", (None, None))
                    gl = tier_gpus.get(dev, []) if dev in (SMALL, LARGE) else []
                    # energy of the serving tier's GPU(s) over the query window: cumulative-counter
                    # delta (reference: power integrated over the window, routing_chatbot_tester.py
                    # :239-254); with tiers sharing a GPU this is that GPU's energy, not a tier share
                    if sampler is not None and gl and marks[0] is not None and marks[1] is not None:
                        e, method = sampler.energy_between(gl, marks[0], marks[1])
                    else:
                        e, method = 0.0, "none"
                    r["energy_mJ"] = round(e, 3)
                    r["energy_method"] = method
                    r["energy_gpus"] = " ".join(str(g) for g in gl)
                    toks, lat = int(r.get("response_tokens") or 0), int(r.get("latency_ms") or 0)
                    ok = dev in (SMALL, LARGE) and toks > 0
                    r["latency_per_token_ms"] = lat / toks if ok else ""
                    r["energy_per_token_mJ"] = e / toks if ok else ""
                    r["start_time"] = r["start_time"].isoformat(sep=" ")
                    r["end_time"] = r["end_time"].isoformat(sep=" ")
                    _append(cfg.output_per_query_csv, hdr_q, r)
                s = summarize(rows, cfg.query_set_name, strategy, cache_mode, int(thr), gpus)
                _append(cfg.output_csv, hdr_s, s)
                summaries.append(s)
                for p in (router.nano, router.orin):
                    try:
                        p.server_manager.stop_server()
                    except Exception:
                        pass
    return summaries


def build_pools_from_arg(kind: str, model: str, small_model: Optional[str], large_model: Optional[str]):
    """Returns (pools, tier_gpus, pool_names)."""
    from ..pools.base import EchoPool
    from ..pools.factory import build_pools
    if kind == "echo":
        return ({SMALL: EchoPool(SMALL, 24), LARGE: EchoPool(LARGE, 96)}, {}, {SMALL: "echo", LARGE: "echo"})
    if kind == "gpu":  # BASELINE config 2: one model on one GPU serves both tiers
        spec = {SMALL: {"model": model, "device": "cuda:0", "max_new_tokens": 128, "share": "main"},
                LARGE: {"model": model, "device": "cuda:0", "max_new_tokens": 384, "temperature": 0.8, "top_k": 40,
                        "top_p": 0.9, "share": "main"}}
        return build_pools(spec), {SMALL: [0], LARGE: [0]}, {SMALL: model, LARGE: model}
    if kind == "gpu2":  # BASELINE config 3: small and large models on two GPUs
        sm, lg = small_model or "llama-3.2-1b", large_model or "llama-3-8b"
        spec = {SMALL: {"model": sm, "device": "cuda:0", "max_new_tokens": 128},
                LARGE: {"model": lg, "device": "cuda:1", "max_new_tokens": 384, "temperature": 0.8, "top_k": 40,
                        "top_p": 0.9}}
        return build_pools(spec), {SMALL: [0], LARGE: [1]}, {SMALL: sm, LARGE: lg}
    from ..config import load_config_file
    spec = {k: v for k, v in load_config_file(kind).items() if not k.startswith("_")}
    tg = {}
    for tier, s in spec.items():
        dev = s.get("device", "cuda:0")
        tg[tier] = s.get("gpus") or ([int(dev.split(":")[1])] if ":" in dev else [0])
    return build_pools(spec), tg, {t: s.get("model", s.get("kind", "")) for t, s in spec.items()}


def parse_args(argv=None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description="routing benchmark (reference CSV schemas)")
    p.add_argument("--query-set", required=True)
    p.add_argument("--thresholds", nargs="+", type=int, default=[4000])
    p.add_argument("--fixed-threshold", type=int, default=None)
    p.add_argument("--strategies", nargs="+", default=["token", "heuristic", "semantic", "hybrid"])
    p.add_argument("--cache-modes", nargs="+", default=["off"], choices=["off", "on"])
    p.add_argument("--output-csv", default="benchmark_results.csv")
    p.add_argument("--output-per-query-csv", default="benchmark_per_query.csv")
    p.add_argument("--pools", default="echo", help="echo | gpu | gpu2 | topology JSON/YAML")
    p.add_argument("--model", default="tinyllama-1.1b")
    p.add_argument("--small-model", default=None)
    p.add_argument("--large-model", default=None)
    p.add_argument("--power-hz", type=float, default=10.0)
    p.add_argument("--no-power", action="store_true")
    p.add_argument("--resume", action="store_true", help="append; skip experiments already summarised")
    # accepted for CLI compatibility with the reference; no SSH hop exists on one node
    for flag in ("--nano-ip", "--orin-ip", "--nano-ssh-user", "--orin-ssh-user"):
        p.add_argument(flag, default=None)
    p.add_argument("--nano-ssh-port", type=int, default=22)
    p.add_argument("--orin-ssh-port", type=int, default=22)
    return p.parse_args(argv)


def main(argv=None) -> List[Dict[str, Any]]:
    a = parse_args(argv)
    if a.query_set not in query_sets:
        raise ValueError(f"Unknown query set: {a.query_set}. Available: {list(query_sets)}")
    items = normalize_query_set(query_sets[a.query_set])
    cfg = RunConfig(a.query_set, a.thresholds, a.strategies, a.cache_modes,
                    a.fixed_threshold if a.fixed_threshold is not None else a.thresholds[-1],
                    a.output_csv, a.output_per_query_csv, a.resume)
    if not a.resume:
        for pth in (cfg.output_csv, cfg.output_per_query_csv):
            if os.path.exists(pth):
                os.remove(pth)
    pools, tier_gpus, names = build_pools_from_arg(a.pools, a.model, a.small_model, a.large_model)
    sampler = None
    if not a.no_power and tier_gpus:
        sampler = PowerSampler(sorted({g for v in tier_gpus.values() for g in v}), hz=a.power_hz).start()
    try:
        return run_experiment(items, cfg, pools, tier_gpus, sampler, names)
    finally:
        if sampler:
            sampler.stop()


if __name__ == "__main__":
    main()
