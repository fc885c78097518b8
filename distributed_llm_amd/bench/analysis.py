"""Results analysis (the reference's ``results_analysis.ipynb`` as a module + CLI).

Reference: the notebook loads ``final_results.csv`` (results_analysis.ipynb:463), derives seconds,
joules, s/token and J/token per device (``derive_metrics`` :679-700) and plots latency / energy /
power / per-token costs against the context threshold (:731, :1099, :1148, :1193, :1238).  Here:

  * ``load_legacy``   — read the legacy ``final_results.csv`` schema (bench/legacy_harness.py);
  * ``load_summary``  — read the new harness summary CSV (bench/harness.py SUMMARY_HEADERS);
  * ``derive_metrics``— the notebook's derived columns plus routed tok/s and mean s/query;
  * ``compare``       — per query set, our best routed tok/s and mean s/query against the published
                        table (embedded below);
  * plots are written only when matplotlib is importable (it is not in this image); the markdown
    tables carry the same series.

CLI: ``python -m distributed_llm_amd.bench.analysis final_results.csv [--summary benchmark_results.csv]
[--markdown report.md]``.
"""
from __future__ import annotations

import argparse
import csv
import statistics
from typing import Dict, List, Optional, Sequence

from .query_sets import query_sets

# (query set, threshold, nano lat s, nano tok, nano J/tok, orin lat s, orin tok, orin J/tok)
# — BASELINE.md "Full table" (results_analysis.ipynb:373-451).
PUBLISHED = [
    ("general_knowledge", 100, 922.2, 986, 1.36, 176.0, 4361, 0.377),
    ("general_knowledge", 200, 291.0, 380, 4.82, 184.0, 4639, 0.374),
    ("general_knowledge", 400, 548.4, 607, 5.44, 171.1, 4263, 0.376),
    ("general_knowledge", 800, 1196.4, 899, 8.04, 169.7, 4212, 0.378),
    ("general_knowledge", 1200, 1609.8, 1355, 7.09, 214.9, 4290, 0.408),
    ("general_knowledge", 1800, 2556.9, 2193, 7.02, 172.2, 4179, 0.386),
    ("general_knowledge", 2400, 6737.5, 2491, 16.22, 114.4, 2720, 0.389),
    ("general_knowledge", 3200, 6129.7, 4289, 10.82, 136.2, 3252, 0.650),
    ("general_knowledge", 4000, 11042.4, 3773, 18.00, 30.1, 618, 0.413),
    ("technical_coding", 200, 581.9, 745, 4.60, 252.3, 6377, 0.374),
    ("technical_coding", 400, 517.2, 713, 4.53, 237.7, 6014, 0.376),
    ("technical_coding", 800, 1595.7, 1459, 6.89, 240.0, 6002, 0.379),
    ("technical_coding", 1200, 1036.5, 1292, 4.85, 237.8, 5841, 0.386),
    ("technical_coding", 1800, 2783.2, 2195, 7.67, 206.1, 5145, 0.376),
    ("technical_coding", 2400, 3429.6, 2663, 7.83, 203.3, 5045, 0.382),
    ("technical_coding", 3200, 7407.3, 5868, 8.05, 215.1, 5346, 0.382),
    ("technical_coding", 4000, 7396.5, 4221, 10.98, 137.5, 3311, 0.386),
    ("personal_health", 200, 494.4, 582, 5.04, 241.7, 5306, 0.398),
    ("personal_health", 400, 486.7, 633, 4.84, 242.6, 5437, 0.396),
    ("personal_health", 800, 1018.3, 788, 8.10, 315.0, 5118, 0.612),
    ("personal_health", 1200, 1722.6, 1222, 8.58, 212.3, 5170, 0.387),
    ("personal_health", 1800, 2962.2, 1957, 9.43, 191.2, 4615, 0.388),
    ("personal_health", 2400, 4415.6, 3876, 7.29, 194.3, 4661, 0.389),
    ("personal_health", 3200, 5327.2, 3592, 9.42, 183.5, 4404, 0.390),
    ("personal_health", 4000, 7158.9, 4931, 9.22, 187.6, 4596, 0.384),
]


def published_rows() -> List[Dict[str, float]]:
    out = []
    for qs, thr, nl, nt, nj, ol, ot, oj in PUBLISHED:
        out.append({"query_set": qs, "threshold": thr,
                    "nano_latency_ms": nl * 1000.0, "nano_energy_mJ": nj * nt * 1000.0, "nano_tokens": nt,
                    "orin_latency_ms": ol * 1000.0, "orin_energy_mJ": oj * ot * 1000.0, "orin_tokens": ot})
    return out


def _f(v) -> float:
    try:
        return float(v)
    except (TypeError, ValueError):
        return 0.0


def load_legacy(path: str) -> List[Dict[str, float]]:
    """Legacy ``final_results.csv`` (reference src/tests/chatbot_tester.py:270-272)."""
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append({"query_set": r["Query Set"], "threshold": int(_f(r["Context Threshold"])),
                         "nano_latency_ms": _f(r["Nano Latency (ms)"]), "nano_energy_mJ": _f(r["Nano Energy (mJ)"]),
                         "nano_tokens": int(_f(r["Nano Tokens Generated"])),
                         "orin_latency_ms": _f(r["Orin Latency (ms)"]), "orin_energy_mJ": _f(r["Orin Energy (mJ)"]),
                         "orin_tokens": int(_f(r["Orin Tokens Generated"]))})
    return rows


def load_summary(path: str) -> List[Dict[str, float]]:
    """New-harness summary CSV (reference src/tests/routing_chatbot_tester.py:323-332 + extras)."""
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append({"query_set": r["query_set"], "threshold": int(_f(r["token_threshold"])),
                         "strategy": r.get("strategy", ""), "cache_mode": r.get("cache_mode", ""),
                         "routing_accuracy": _f(r.get("routing_accuracy")),
                         "nano_latency_ms": _f(r["nano_total_latency_ms"]),
                         "nano_energy_mJ": _f(r["nano_total_energy_mJ"]),
                         "nano_tokens": int(_f(r["nano_total_tokens"])),
                         "orin_latency_ms": _f(r["orin_total_latency_ms"]),
                         "orin_energy_mJ": _f(r["orin_total_energy_mJ"]),
                         "orin_tokens": int(_f(r["orin_total_tokens"])),
                         "gpus": int(_f(r.get("gpus", 0))) or None,
                         "p50_latency_ms": _f(r.get("p50_latency_ms")) or None})
    return rows


def derive_metrics(rows: Sequence[Dict[str, float]]) -> List[Dict[str, float]]:
    """The notebook's derive_metrics (:679-700): s, J, s/token, J/token per device, plus the
    routed aggregate (tok/s over the summed latency, mean s/query for the set's query count)."""
    out = []
    for r in rows:
        d = dict(r)
        for dev in ("nano", "orin"):
            s = r[f"{dev}_latency_ms"] / 1000.0
            j = r[f"{dev}_energy_mJ"] / 1000.0
            t = r[f"{dev}_tokens"]
            d[f"{dev}_s"] = s
            d[f"{dev}_J"] = j
            d[f"{dev}_s_per_token"] = s / t if t else None
            d[f"{dev}_J_per_token"] = j / t if t else None
            d[f"{dev}_avg_power_W"] = j / s if s > 0 else None
        tot_s = d["nano_s"] + d["orin_s"]
        tot_t = r["nano_tokens"] + r["orin_tokens"]
        n_q = len(query_sets.get(r["query_set"], [])) or 1
        d["total_s"] = tot_s
        d["total_tokens"] = tot_t
        d["routed_tok_s"] = tot_t / tot_s if tot_s > 0 else None
        d["mean_s_per_query"] = tot_s / n_q
        out.append(d)
    return out


def best_by_set(rows: Sequence[Dict[str, float]]) -> Dict[str, Dict[str, float]]:
    best: Dict[str, Dict[str, float]] = {}
    for r in derive_metrics(rows):
        cur = best.get(r["query_set"])
        if r["routed_tok_s"] is not None and (cur is None or r["routed_tok_s"] > cur["routed_tok_s"]):
            best[r["query_set"]] = r
    return best


def compare(ours: Sequence[Dict[str, float]]) -> List[Dict[str, object]]:
    """Per query set: best routed tok/s and mean s/query, ours vs published."""
    pub, mine = best_by_set(published_rows()), best_by_set(ours)
    out = []
    for qs in sorted(set(pub) | set(mine)):
        p, m = pub.get(qs), mine.get(qs)
        row: Dict[str, object] = {"query_set": qs}
        if p:
            row.update(pub_threshold=p["threshold"], pub_tok_s=round(p["routed_tok_s"], 2),
                       pub_s_per_query=round(p["mean_s_per_query"], 1))
        if m:
            row.update(our_threshold=m["threshold"], our_tok_s=round(m["routed_tok_s"], 2),
                       our_s_per_query=round(m["mean_s_per_query"], 3))
        if p and m and p["routed_tok_s"]:
            row["tok_s_speedup"] = round(m["routed_tok_s"] / p["routed_tok_s"], 1)
            row["latency_speedup"] = round(p["mean_s_per_query"] / max(m["mean_s_per_query"], 1e-9), 1)
        out.append(row)
    return out


def markdown_table(rows: Sequence[Dict[str, object]], cols: Optional[Sequence[str]] = None) -> str:
    if not rows:
        return "(no rows)\n"
    cols = list(cols or rows[0].keys())

    def fmt(v):
        if v is None:
            return "—"
        if isinstance(v, float):
            return f"{v:.4g}"
        return str(v)
    lines = ["| " + " | ".join(cols) + " |", "|" + "---|" * len(cols)]
    for r in rows:
        lines.append("| " + " | ".join(fmt(r.get(c)) for c in cols) + " |")
    return "\n".join(lines) + "\n"


DERIVED_COLS = ["query_set", "threshold", "nano_s", "nano_tokens", "nano_s_per_token", "nano_J_per_token",
                "orin_s", "orin_tokens", "orin_s_per_token", "orin_J_per_token", "routed_tok_s", "mean_s_per_query"]


def plot(rows: Sequence[Dict[str, float]], out_prefix: str) -> List[str]:
    """Notebook plots (latency / energy / power / per-token vs threshold) if matplotlib exists."""
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        return []
    d = derive_metrics(rows)
    written = []
    for key, label in (("s", "latency (s)"), ("J", "energy (J)"), ("avg_power_W", "avg power (W)"),
                       ("s_per_token", "latency per token (s)"), ("J_per_token", "energy per token (J)")):
        fig, ax = plt.subplots()
        for qs in sorted({r["query_set"] for r in d}):
            rs = sorted((r for r in d if r["query_set"] == qs), key=lambda r: r["threshold"])
            for dev in ("nano", "orin"):
                ax.plot([r["threshold"] for r in rs], [r[f"{dev}_{key}"] or 0 for r in rs], marker="o",
                        label=f"{qs} {dev}")
        ax.set_xlabel("context threshold")
        ax.set_ylabel(label)
        ax.legend(fontsize=6)
        path = f"{out_prefix}_{key}.png"
        fig.savefig(path, dpi=120)
        plt.close(fig)
        written.append(path)
    return written


def main(argv=None) -> str:
    ap = argparse.ArgumentParser()
    ap.add_argument("legacy_csv", nargs="?", default=None, help="final_results.csv (legacy schema)")
    ap.add_argument("--summary", default=None, help="benchmark_results.csv (new harness summary)")
    ap.add_argument("--markdown", default=None)
    ap.add_argument("--plots", default=None, help="output prefix for PNG plots (needs matplotlib)")
    a = ap.parse_args(argv)
    rows: List[Dict[str, float]] = []
    if a.legacy_csv:
        rows += load_legacy(a.legacy_csv)
    if a.summary:
        rows += load_summary(a.summary)
    parts = ["## Derived metrics (ours)\n", markdown_table(derive_metrics(rows), DERIVED_COLS) if rows else "(none)\n",
             "\n## Best routed throughput per query set: ours vs published\n", markdown_table(compare(rows))]
    if a.summary:
        srows = load_summary(a.summary)
        by = {}
        for r in derive_metrics(srows):
            by.setdefault((r.get("strategy"), r.get("cache_mode")), []).append(r)
        agg = [{"strategy": k[0], "cache_mode": k[1], "runs": len(v),
                "mean_routing_accuracy": round(statistics.mean(x["routing_accuracy"] for x in v), 3),
                "mean_routed_tok_s": round(statistics.mean(x["routed_tok_s"] or 0 for x in v), 2)}
               for k, v in sorted(by.items())]
        parts += ["\n## Per strategy (new harness)\n", markdown_table(agg)]
    text = "".join(parts)
    if a.plots and rows:
        plot(rows, a.plots)
    if a.markdown:
        with open(a.markdown, "w") as f:
            f.write(text)
    print(text)
    return text


if __name__ == "__main__":
    main()
