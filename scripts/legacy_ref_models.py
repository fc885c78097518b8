"""The reference's published protocol with the reference's own model pair on ONE MI355X.

Legacy harness (``bench/legacy_harness.py`` = ``src/tests/chatbot_tester.py``, the producer of
every published number in BASELINE.md) over the three query sets: phi3-mini serves the small
(Nano) tier greedily, Llama-3-8B the large (Orin) tier with Ollama-default sampling, as
``src/devices/nano_api.py:15-21`` / ``orin_api.py:17-18`` do (random-init bf16 weights here; the
reference runs Ollama's 4-bit weights).  Token-router thresholds (the published trend) 200 / 400.
Writes ``final_results.csv`` rows plus a per-tier JSON summary line per query set, with tokens
counted two ways: as the reference does (TokenCounter on the returned text) and as decoded.

Usage: python scripts/legacy_ref_models.py <out_dir>
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_llm_amd.bench.harness import build_pools_from_arg  # noqa: E402
from distributed_llm_amd.bench.legacy_harness import run_legacy  # noqa: E402
from distributed_llm_amd.bench.power import PowerSampler  # noqa: E402
from distributed_llm_amd.config import LARGE, SMALL  # noqa: E402

TOPO = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "distributed_llm_amd", "data", "topologies", "reference_models_1gpu.json")


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/legacy_ref"
    os.makedirs(out, exist_ok=True)
    thresholds = [int(x) for x in os.environ.get("THRESHOLDS", "200 400").split()]
    t = time.perf_counter()
    pools, tier_gpus, names = build_pools_from_arg(TOPO, "", None, None)
    for p in pools.values():
        eng = getattr(p, "engine", None)
        if eng is not None and eng.on_gpu:
            eng.capture_all(max_bs=8)
    print(json.dumps({"setup_s": round(time.perf_counter() - t, 1), "pools": names}), flush=True)
    sampler = PowerSampler(sorted({g for v in tier_gpus.values() for g in v}), hz=10.0).start()
    try:
        for qs in ("general_knowledge", "technical_coding", "personal_health"):
            gen0 = {d: p.engine.stats()["decode_tokens"] for d, p in pools.items()}
            res = run_legacy(qs, thresholds, pools, tier_gpus, sampler, threshold_routing=True,
                             output_file=os.path.join(out, "final_results.csv"))
            gen = {d: p.engine.stats()["decode_tokens"] - gen0[d] for d, p in pools.items()}
            for thr, r in res.items():
                lat = (r[SMALL][0] + r[LARGE][0]) / 1000.0
                tok = r[SMALL][3] + r[LARGE][3]
                print(json.dumps({"query_set": qs, "threshold": thr, "total_latency_s": round(lat, 2),
                                  "reference_counted_tokens": tok,
                                  "routed_tok_s_reference_counting": round(tok / max(lat, 1e-9), 2),
                                  "nano_s": r[SMALL][0] / 1000.0, "orin_s": r[LARGE][0] / 1000.0,
                                  "nano_W": r[SMALL][2], "orin_W": r[LARGE][2]}), flush=True)
            print(json.dumps({"query_set": qs, "decoded_tokens_all_thresholds": gen}), flush=True)
    finally:
        sampler.stop()


if __name__ == "__main__":
    main()
