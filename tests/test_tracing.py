"""Span tracer (utils/tracing.py): Chrome trace export, thread safety, no-op when disabled, and the
engine / orchestrator spans of one routed request on CPU."""
import json
import threading

import pytest

from distributed_llm_amd.utils.tracing import Tracer, tracer


def test_disabled_tracer_records_nothing():
    t = Tracer()
    with t.span("x", a=1) as args:
        args["b"] = 2
    t.counter("c", v=1.0)
    t.instant("i")
    assert t.events() == []


def test_spans_nest_and_export(tmp_path):
    t = Tracer().enable(str(tmp_path / "trace.json"))
    with t.span("outer", "cat", k=1) as a:
        with t.span("inner"):
            pass
        a["extra"] = "v"
    t.counter("batch", running=3)
    t.instant("mark")
    with t.gpu_span("gpu_block"):   # no GPU here: falls back to a host span
        pass
    path = t.dump()
    doc = json.load(open(path))
    evs = doc["traceEvents"]
    by = {e["name"]: e for e in evs}
    assert by["outer"]["ph"] == "X" and by["outer"]["args"] == {"k": 1, "extra": "v"}
    o, i = by["outer"], by["inner"]
    assert o["ts"] <= i["ts"] and i["ts"] + i["dur"] <= o["ts"] + o["dur"] + 1e-3
    assert by["batch"]["ph"] == "C" and by["batch"]["args"] == {"running": 3}
    assert by["mark"]["ph"] == "i"
    assert "gpu_block" in by
    assert any(e["ph"] == "M" for e in evs)
    s = t.summary()
    assert s["outer"]["count"] == 1 and s["outer"]["total_ms"] >= s["inner"]["total_ms"]


def test_bounded_and_thread_safe():
    t = Tracer(max_events=1000).enable()

    def work():
        for _ in range(500):
            with t.span("w"):
                pass

    ts = [threading.Thread(target=work) for _ in range(8)]
    for th in ts:
        th.start()
    for th in ts:
        th.join()
    assert len(t.events()) == 1000


def test_routed_request_spans(tmp_path):
    from distributed_llm_amd.config import LARGE, SMALL
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    from distributed_llm_amd.orchestrator import Router
    from distributed_llm_amd.pools.base import EnginePool

    eng = LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=4, seed=0)
    pools = {SMALL: EnginePool(SMALL, eng, max_new_tokens=4), LARGE: EnginePool(LARGE, eng, max_new_tokens=4)}
    r = Router("token", config={"cache_enabled": False}, pools=pools)
    tracer.clear()
    tracer.enable(str(tmp_path / "routed.json"))
    try:
        payload, toks, dev = r.route_query([{"role": "user", "content": "hello there"}])
    finally:
        tracer.disable()
    assert payload["ok"]
    names = {e["name"] for e in tracer.events()}
    assert {"route.decide", "pool.process", "engine.prefill", "request.queue", "request.prefill",
            "request.decode"} <= names
    req = [e for e in tracer.events() if e["name"] == "request.decode"][0]
    assert req["args"]["generated"] == 4 and req["tid"].startswith("req ")
    dec = [e for e in tracer.events() if e["name"] == "route.decide"][0]
    assert dec["args"]["device"] == dev
    doc = json.load(open(tracer.dump()))
    assert doc["traceEvents"]
    tracer.clear()


@pytest.mark.gpu
def test_gpu_span_times_device_work():
    import torch
    t = Tracer().enable()
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    with t.gpu_span("mm", n=4096):
        for _ in range(8):
            a = a @ a.t() * 1e-3
    ev = [e for e in t.events() if e["name"] == "mm"]
    gpu = [e for e in ev if str(e["tid"]).startswith("gpu:")]
    host = [e for e in ev if not str(e["tid"]).startswith("gpu:")]
    assert len(gpu) == 1 and len(host) == 1
    # 8 x 137 GFLOP takes well over 100 us on the device even at peak
    assert gpu[0]["dur"] > 100.0 and gpu[0]["args"] == {"n": 4096}
    assert "mm[gpu]" in t.summary()
