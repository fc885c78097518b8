"""Legacy context-threshold sweep -> ``final_results.csv`` (the schema of the reference's ONLY
published numbers).

Reference: ``src/tests/chatbot_tester.py`` (``run_test`` :108-138, ``calculate_energy``
:207-251, ``save_results`` :255-284; header :270-272).  Same loop: perf strategy, routing cache and
response cache off, failover on; for each threshold ``Router.set_threshold(t)`` and a fresh
conversation over the query set; per threshold and tier: total latency (ms), energy (mJ), average
power (W = mJ / ms) and generated tokens.

Energy: the reference sums 1 Hz mW samples (= mJ at 1 Hz) inside each query window.  Here each
query's energy is the GPU energy-counter delta over its window (``PowerSampler.mark`` /
``energy_between``; trapezoid over the interpolated power trace where no counter exists), so
sub-second queries are not read as 0 mJ.  Note: ``set_threshold`` only
moves the routing-exception fallback, so — as in the reference's current code — the threshold axis
does not change perf routing; ``--threshold-routing`` instead sweeps the token router's threshold,
which is what the published table's trend reflects.
"""
from __future__ import annotations

import argparse
import csv
import os
from datetime import datetime
from typing import Dict, List, Optional, Sequence

from ..config import LARGE, SMALL
from .power import PowerSampler
from .query_sets import normalize_query_set, query_sets

LEGACY_HEADER = ["Query Set", "Context Threshold",
                 "Nano Latency (ms)", "Nano Energy (mJ)", "Nano Avg Power (W)", "Nano Tokens Generated",
                 "Orin Latency (ms)", "Orin Energy (mJ)", "Orin Avg Power (W)", "Orin Tokens Generated"]


def run_legacy(query_set: str, thresholds: Sequence[int], pools, tier_gpus: Dict[str, List[int]],
               sampler: Optional[PowerSampler] = None, threshold_routing: bool = False,
               output_file: str = "final_results.csv") -> Dict[int, Dict[str, List[float]]]:
    from ..orchestrator import Router
    items = [it.text for it in normalize_query_set(query_sets[query_set])]
    log = []
    for thr in thresholds:
        if threshold_routing:
            cfg = {"cache_enabled": False, "enable_response_cache": False, "enable_failover": True,
                   "token_threshold": thr}
            router = Router(strategy="token", config=cfg, threshold_fallback=thr, pools=pools)
        else:
            cfg = {"cache_enabled": False, "enable_response_cache": False, "enable_failover": True}
            router = Router(strategy="perf", config=cfg, threshold_fallback=100, pools=pools)
            router.set_threshold(thr)
        history = []
        for q in items:
            history.append({"role": "user", "content": q})
            m0 = sampler.mark() if sampler is not None else None
            t0 = datetime.now()
            payload, ntok, dev = router.route_query(history)
            t1 = datetime.now()
            m1 = sampler.mark() if sampler is not None else None
            history.append({"role": "assistant", "content": payload.get("response", "")})
            log.append((thr, dev, t0, t1, int(ntok), m0, m1))
    results: Dict[int, Dict[str, List[float]]] = {}
    for thr, dev, t0, t1, ntok, m0, m1 in log:
        r = results.setdefault(thr, {SMALL: [0, 0.0, 0.0, 0], LARGE: [0, 0.0, 0.0, 0]})
        if dev not in r:
            continue
        e = 0.0
        if sampler is not None and m0 is not None and m1 is not None:
            e = sampler.energy_between(tier_gpus.get(dev, []), m0, m1)[0]
        r[dev][0] += round((t1 - t0).total_seconds() * 1000)
        r[dev][1] += e
        r[dev][3] += ntok
    for thr in results:
        for dev in (SMALL, LARGE):
            lat, e = results[thr][dev][0], results[thr][dev][1]
            results[thr][dev][2] = round(e / lat, 3) if lat > 0 else 0
    new = not os.path.exists(output_file)
    with open(output_file, "a", newline="") as f:
        w = csv.writer(f)
        if new:
            w.writerow(LEGACY_HEADER)
        for thr, d in results.items():
            w.writerow([query_set, thr, d[SMALL][0], round(d[SMALL][1], 3), d[SMALL][2], d[SMALL][3],
                        d[LARGE][0], round(d[LARGE][1], 3), d[LARGE][2], d[LARGE][3]])
    return results


def main(argv=None):
    from .harness import build_pools_from_arg
    ap = argparse.ArgumentParser()
    ap.add_argument("--query-set", default="personal_health")
    ap.add_argument("--thresholds", nargs="+", type=int, default=[4000])
    ap.add_argument("--pools", default="echo")
    ap.add_argument("--model", default="tinyllama-1.1b")
    ap.add_argument("--output", default="final_results.csv")
    ap.add_argument("--threshold-routing", action="store_true")
    ap.add_argument("--no-power", action="store_true")
    a = ap.parse_args(argv)
    pools, tier_gpus, _ = build_pools_from_arg(a.pools, a.model, None, None)
    sampler = None
    if not a.no_power and tier_gpus:
        sampler = PowerSampler(sorted({g for v in tier_gpus.values() for g in v}), hz=10.0).start()
    try:
        return run_legacy(a.query_set, a.thresholds, pools, tier_gpus, sampler, a.threshold_routing, a.output)
    finally:
        if sampler:
            sampler.stop()


if __name__ == "__main__":
    main()
