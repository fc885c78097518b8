"""Benchmark harness: reference CSV schemas (column names and order), experiment sweep semantics,
resume, legacy final_results.csv, power-log parsing, CLI REPL — on echo pools (BASELINE config 1)."""
import csv
import io
import os
from datetime import datetime, timedelta

from distributed_llm_amd.bench import harness, legacy_harness, power
from distributed_llm_amd.config import LARGE, SMALL
from distributed_llm_amd.pools.base import EchoPool

REF_SUMMARY = ["query_set", "strategy", "cache_mode", "token_threshold", "routing_accuracy",
               "nano_total_latency_ms", "nano_total_energy_mJ", "nano_avg_power_mW", "nano_total_tokens",
               "nano_latency_per_token_ms", "nano_energy_per_token_mJ",
               "orin_total_latency_ms", "orin_total_energy_mJ", "orin_avg_power_mW", "orin_total_tokens",
               "orin_latency_per_token_ms", "orin_energy_per_token_mJ",
               "overall_total_latency_ms", "overall_total_energy_mJ", "overall_total_tokens",
               "overall_latency_per_token_ms", "overall_energy_per_token_mJ"]
REF_PER_QUERY = ["query_set", "strategy", "cache_mode", "token_threshold", "query_index", "query_text",
                 "expected_device", "device_used", "cache_hit", "routing_method", "routing_confidence",
                 "routing_reasoning", "routing_overhead_ms", "start_time", "end_time", "latency_ms",
                 "response_tokens", "energy_mJ", "latency_per_token_ms", "energy_per_token_mJ"]


def test_harness_schema_and_sweep(tmp_path):
    out, pq = str(tmp_path / "s.csv"), str(tmp_path / "q.csv")
    harness.main(["--query-set", "general_knowledge", "--thresholds", "100", "1000",
                  "--strategies", "token", "heuristic", "--cache-modes", "off", "on",
                  "--output-csv", out, "--output-per-query-csv", pq, "--pools", "echo", "--no-power"])
    with open(out) as f:
        rows = list(csv.reader(f))
    assert rows[0][:len(REF_SUMMARY)] == REF_SUMMARY
    assert rows[0][len(REF_SUMMARY):] == harness.SUMMARY_EXTRA
    # token sweeps 2 thresholds x 2 cache modes; heuristic runs once per cache mode at the last threshold
    keys = [(r[1], r[2], r[3]) for r in rows[1:]]
    assert keys == [("token", "off", "100"), ("token", "off", "1000"), ("token", "on", "100"),
                    ("token", "on", "1000"), ("heuristic", "off", "1000"), ("heuristic", "on", "1000")]
    with open(pq) as f:
        q = list(csv.DictReader(f))
    assert list(q[0].keys())[:len(REF_PER_QUERY)] == REF_PER_QUERY
    assert len(q) == 6 * 12
    heur = [r for r in q if r["strategy"] == "heuristic" and r["cache_mode"] == "off"]
    assert heur[0]["device_used"] == "nano" and heur[0]["routing_method"] == "heuristic"
    acc = [r for r in rows[1:] if r[1] == "heuristic" and r[2] == "off"][0][4]
    assert 0.0 <= float(acc) <= 1.0


def test_heuristic_accuracy_goldens():
    """SURVEY §2.9 probe goldens: per-query heuristic accuracy 0.75 / 0.80 / 1.00."""
    from distributed_llm_amd.bench.query_sets import normalize_query_set, query_sets
    from distributed_llm_amd.config import BENCHMARK_CFG
    from distributed_llm_amd.router.query_router import QueryRouter
    qr = QueryRouter("heuristic", dict(BENCHMARK_CFG))
    for name, want in (("general_knowledge", 0.75), ("technical_coding", 0.80), ("personal_health", 1.00)):
        items = normalize_query_set(query_sets[name])
        acc = sum(qr.route_query(i.text).device == i.expected_device for i in items) / len(items)
        assert abs(acc - want) < 1e-9, name


def test_harness_resume(tmp_path):
    out, pq = str(tmp_path / "s.csv"), str(tmp_path / "q.csv")
    args = ["--query-set", "technical_coding", "--strategies", "heuristic", "--output-csv", out,
            "--output-per-query-csv", pq, "--pools", "echo", "--no-power"]
    harness.main(args)
    harness.main(args + ["--strategies", "heuristic", "token", "--resume"])
    with open(out) as f:
        rows = list(csv.reader(f))
    assert [r[1] for r in rows[1:]] == ["heuristic", "token"]
    # a different query set with the same (strategy, cache, threshold) is NOT skipped on resume
    args2 = [a if a != "technical_coding" else "personal_health" for a in args]
    harness.main(args2 + ["--resume"])
    with open(out) as f:
        rows = list(csv.reader(f))
    assert [(r[0], r[1]) for r in rows[1:]] == [("technical_coding", "heuristic"), ("technical_coding", "token"),
                                                ("personal_health", "heuristic")]


def test_legacy_final_results(tmp_path):
    out = str(tmp_path / "final_results.csv")
    pools = {SMALL: EchoPool(SMALL, 5), LARGE: EchoPool(LARGE, 50)}
    res = legacy_harness.run_legacy("personal_health", [100, 4000], pools, {}, None, threshold_routing=True,
                                    output_file=out)
    with open(out) as f:
        rows = list(csv.reader(f))
    assert rows[0] == legacy_harness.LEGACY_HEADER
    assert len(rows) == 3 and rows[1][0] == "personal_health" and rows[1][1] == "100"
    # a higher token threshold sends more turns to the small tier (the published table's trend)
    assert res[4000][SMALL][3] >= res[100][SMALL][3]


def test_power_log_roundtrip(tmp_path):
    p = tmp_path / "power.log"
    t0 = datetime(2026, 1, 1, 12, 0, 0)
    lines = [f"{(t0 + timedelta(seconds=i)).strftime(power.TS_FMT)}: {1000 * (i + 1)}" for i in range(5)]
    p.write_text("\n".join(lines + ["garbage line", "2026-01-01 12:00:09: notanumber"]) + "\n")
    data = power.parse_power_log(str(p))
    assert len(data) == 5
    # left Riemann over [0, 4] s: 1000 + 2000 + 3000 + 4000 mW*s
    assert power.energy_for_window(data, t0, t0 + timedelta(seconds=4)) == 10000.0
    assert power.energy_sum_1hz(data, t0, t0 + timedelta(seconds=4)) == 15000.0


def test_power_sampler_degrades_without_gpu():
    s = power.PowerSampler(gpus=[0], hz=5).start()
    s.stop()
    assert s.energy_mj([0], datetime.now(), datetime.now()) == 0.0
    m0, m1 = s.mark(), s.mark()
    assert s.energy_between([0], m0, m1) == (0.0, "none")


def test_trapezoid_energy_sub_sample_windows():
    """A window shorter than the sample period reads interpolated power x duration (the old
    in-window sample sum read 0 mJ: profiles/r2_harness_1gpu/benchmark_results.csv)."""
    t0 = datetime(2026, 1, 1, 12, 0, 0)
    trace = [(t0 + timedelta(seconds=i), 100_000 + 10_000 * i) for i in range(6)]   # mW, 1 Hz ramp
    # 100 ms window between two samples: power 105,000 -> 106,000 mW
    w0, w1 = t0 + timedelta(seconds=0.5), t0 + timedelta(seconds=0.6)
    e = power.energy_for_window_trapz(trace, w0, w1)
    assert abs(e - 0.1 * 105_500) < 1e-6
    assert power.energy_for_window(dict(trace), w0, w1) == 0.0          # the reference's left-Riemann
    # window spanning samples: exact integral of the linear ramp (boundary segments included)
    e = power.energy_for_window_trapz(trace, t0 + timedelta(seconds=0.25), t0 + timedelta(seconds=3.75))
    exact = 3.5 * 100_000 + 10_000 * (3.75 ** 2 - 0.25 ** 2) / 2
    assert abs(e - exact) < 1e-6
    # outside the trace: held at the edge value
    e = power.energy_for_window_trapz(trace, t0 - timedelta(seconds=1), t0)
    assert abs(e - 100_000) < 1e-6
    assert power.energy_for_window_trapz([], w0, w1) == 0.0


def test_energy_counter_marks_preferred_over_trace():
    """With an energy counter the per-query energy is the counter delta; a GPU without one falls
    back to the interpolated trace."""
    class Fake(power.PowerSampler):
        def __init__(self):
            self.hz, self.log_path, self.available = 10.0, None, True
            self._handles = [(0, "h0"), (1, "h1")]
            t0 = datetime(2026, 1, 1)
            self.samples = {0: [], 1: [(t0, 200_000), (t0 + timedelta(seconds=10), 200_000)]}
            self.counter = 1_000.0

        def counter_mj(self, handle):
            return self.counter if handle == "h0" else None

    s = Fake()
    m0 = power.EnergyMark(datetime(2026, 1, 1, 0, 0, 1), {0: 1_000.0, 1: None})
    m1 = power.EnergyMark(datetime(2026, 1, 1, 0, 0, 1, 250_000), {0: 1_230.5, 1: None})
    assert s.energy_between([0], m0, m1) == (230.5, "counter")
    e, how = s.energy_between([1], m0, m1)
    assert how == "trapz" and abs(e - 0.25 * 200_000) < 1e-6
    e, how = s.energy_between([0, 1], m0, m1)
    assert how == "counter" and abs(e - (230.5 + 50_000)) < 1e-6
    mk = s.mark()
    assert mk.counters == {0: 1_000.0, 1: None}


def test_cli_repl():
    from distributed_llm_amd.server.cli import Chatbot
    bot = Chatbot(strategy="heuristic", config={"cache_enabled": False}, pools={SMALL: EchoPool(SMALL, 3),
                                                                                LARGE: EchoPool(LARGE, 9)})
    out = io.StringIO()
    bot.chat(stdin=io.StringIO("Thank you!\nquit\n"), stdout=out)
    assert "Assistant:" in out.getvalue() and "[nano]" in out.getvalue()
    assert len(bot.conversation_history) == 2


def test_analysis_derived_metrics_and_compare(tmp_path):
    """bench.analysis (reference results_analysis.ipynb): published table re-derives BASELINE.md's
    headline numbers, and our CSVs (legacy + summary) load and compare."""
    from distributed_llm_amd.bench import analysis
    pub = analysis.derive_metrics(analysis.published_rows())
    gk200 = [r for r in pub if r["query_set"] == "general_knowledge" and r["threshold"] == 200][0]
    assert abs(gk200["routed_tok_s"] - 10.57) < 0.01          # BASELINE.md best routed tok/s
    assert abs(gk200["mean_s_per_query"] - 39.6) < 0.05        # BASELINE.md best mean s/query
    best = analysis.best_by_set(analysis.published_rows())
    assert best["technical_coding"]["threshold"] == 400 and best["personal_health"]["threshold"] == 400

    legacy = str(tmp_path / "final_results.csv")
    pools = {SMALL: EchoPool(SMALL, 5), LARGE: EchoPool(LARGE, 50)}
    legacy_harness.run_legacy("personal_health", [100, 4000], pools, {}, None, threshold_routing=True,
                              output_file=legacy)
    summ, pq = str(tmp_path / "s.csv"), str(tmp_path / "q.csv")
    harness.main(["--query-set", "general_knowledge", "--strategies", "token", "heuristic",
                  "--output-csv", summ, "--output-per-query-csv", pq, "--pools", "echo", "--no-power"])
    md = str(tmp_path / "report.md")
    text = analysis.main([legacy, "--summary", summ, "--markdown", md])
    assert "personal_health" in text and "general_knowledge" in text and "pub_tok_s" in text
    assert os.path.exists(md)
    rows = analysis.derive_metrics(analysis.load_legacy(legacy))
    assert len(rows) == 2 and all(r["total_tokens"] > 0 for r in rows)
