"""Span tracing for the serving path, exported as Chrome trace-event JSON (chrome://tracing, Perfetto).

The reference has wall-clock timers only (`src/router.py:159-170,236,272`, per-query start/end in
`src/tests/routing_chatbot_tester.py:408-442`). This module adds what SURVEY §5.1 asks
for on top of the per-request queue / TTFT / decode split that `RequestOutput` already carries:

* host spans (`span()`), nested per thread: routing decision, pool dispatch, engine prefill and
  decode steps, with free-form args (batch size, graph bucket, tokens);
* optional GPU spans (`gpu_span()`): a pair of HIP events recorded on the current stream around
  the block; the elapsed GPU time is resolved lazily at `dump()` so recording never synchronises
  the device inside the decode loop;
* counters (`counter()`), e.g. running batch size and free KV blocks per step;
* per-request lifecycle spans (`complete()`): queue wait, prefill until the first token, decode,
  on rotating `req NN` lanes, so each query's latency split is visible next to the engine steps.

Tracing is off unless `DLLM_TRACE=<path>` is set or `enable()` is called; when off every call is
a no-op costing one attribute check. Events go into a bounded deque (`DLLM_TRACE_MAX`, default
1M events) under a lock, so concurrent pool threads can record safely.
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from collections import deque
from typing import Any, Dict, Iterator, List, Optional

__all__ = ["Tracer", "tracer", "span", "gpu_span", "counter", "instant", "enable", "disable", "dump"]


class Tracer:
    def __init__(self, max_events: int = 1_000_000) -> None:
        self.enabled = False
        self.path: Optional[str] = None
        self._ev: deque = deque(maxlen=max_events)
        self._gpu: List[tuple] = []        # (name, cat, tid, host_ts_us, start_evt, end_evt, args)
        self._lock = threading.Lock()
        self._t0 = time.perf_counter()
        self._pid = os.getpid()

    # ------------------------------------------------------------------ control
    def enable(self, path: Optional[str] = None) -> "Tracer":
        self.path = path or self.path
        self.enabled = True
        return self

    def disable(self) -> None:
        self.enabled = False

    def clear(self) -> None:
        with self._lock:
            self._ev.clear()
            self._gpu.clear()

    def _now_us(self) -> float:
        return (time.perf_counter() - self._t0) * 1e6

    # ------------------------------------------------------------------ recording
    @contextlib.contextmanager
    def span(self, name: str, cat: str = "host", **args: Any) -> Iterator[Dict[str, Any]]:
        """Complete ('X') event around the block. The yielded dict can be filled with more args."""
        if not self.enabled:
            yield args
            return
        ts = self._now_us()
        try:
            yield args
        finally:
            ev = {"name": name, "cat": cat, "ph": "X", "ts": ts, "dur": self._now_us() - ts,
                  "pid": self._pid, "tid": threading.get_ident()}
            if args:
                ev["args"] = dict(args)
            with self._lock:
                self._ev.append(ev)

    @contextlib.contextmanager
    def gpu_span(self, name: str, cat: str = "gpu", **args: Any) -> Iterator[Dict[str, Any]]:
        """Host span plus a HIP event pair on the current stream (GPU duration resolved at dump)."""
        if not self.enabled:
            yield args
            return
        import torch
        if not torch.cuda.is_available():
            with self.span(name, cat, **args) as a:
                yield a
            return
        start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = self._now_us()
        start.record()
        try:
            with self.span(name, "host", **args) as a:
                yield a
        finally:
            end.record()
            with self._lock:
                self._gpu.append((name, cat, threading.get_ident(), ts, start, end, dict(args)))

    def complete(self, name: str, t_start: float, t_end: float, cat: str = "request", lane: str = "requests",
                 **args: Any) -> None:
        """Span with explicit ``time.perf_counter()`` bounds on a named lane (per-request lifecycle
        phases recorded after the fact: queue wait, prefill-to-first-token, decode)."""
        if not self.enabled or t_end < t_start:
            return
        ev = {"name": name, "cat": cat, "ph": "X", "ts": (t_start - self._t0) * 1e6,
              "dur": (t_end - t_start) * 1e6, "pid": self._pid, "tid": lane}
        if args:
            ev["args"] = args
        with self._lock:
            self._ev.append(ev)

    def instant(self, name: str, cat: str = "host", **args: Any) -> None:
        if not self.enabled:
            return
        ev = {"name": name, "cat": cat, "ph": "i", "s": "t", "ts": self._now_us(), "pid": self._pid,
              "tid": threading.get_ident()}
        if args:
            ev["args"] = args
        with self._lock:
            self._ev.append(ev)

    def counter(self, name: str, **values: float) -> None:
        if not self.enabled:
            return
        ev = {"name": name, "ph": "C", "ts": self._now_us(), "pid": self._pid, "args": values}
        with self._lock:
            self._ev.append(ev)

    # ------------------------------------------------------------------ export
    def _resolve_gpu(self) -> List[Dict[str, Any]]:
        out = []
        with self._lock:
            pending, self._gpu = self._gpu, []
        for name, cat, tid, ts, s, e, args in pending:
            e.synchronize()
            dur = s.elapsed_time(e) * 1000.0      # ms -> us
            # GPU lane: host enqueue time as the start (HIP event timestamps are on a different clock)
            out.append({"name": name, "cat": cat, "ph": "X", "ts": ts, "dur": dur, "pid": self._pid,
                        "tid": f"gpu:{tid}", "args": args})
        return out

    def events(self) -> List[Dict[str, Any]]:
        gpu = self._resolve_gpu()
        with self._lock:
            evs = list(self._ev)
        evs.extend(gpu)
        with self._lock:
            self._ev.extend(gpu)
        return evs

    def summary(self) -> Dict[str, Dict[str, float]]:
        """Per span name: count, total / mean / max duration in ms."""
        agg: Dict[str, Dict[str, float]] = {}
        for ev in self.events():
            if ev.get("ph") != "X":
                continue
            key = ev["name"] if not str(ev["tid"]).startswith("gpu:") else f"{ev['name']}[gpu]"
            a = agg.setdefault(key, {"count": 0, "total_ms": 0.0, "max_ms": 0.0})
            d = ev["dur"] / 1000.0
            a["count"] += 1
            a["total_ms"] += d
            a["max_ms"] = max(a["max_ms"], d)
        for a in agg.values():
            a["mean_ms"] = a["total_ms"] / max(1, a["count"])
        return agg

    def dump(self, path: Optional[str] = None) -> Optional[str]:
        path = path or self.path
        if not path:
            return None
        evs = self.events()
        meta = [{"name": "process_name", "ph": "M", "pid": self._pid,
                 "args": {"name": f"dllm rank {os.environ.get('RANK', '0')}"}}]
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump({"traceEvents": meta + evs, "displayTimeUnit": "ms"}, f)
        return path


tracer = Tracer(int(os.environ.get("DLLM_TRACE_MAX", "1000000")))
if os.environ.get("DLLM_TRACE"):
    _p = os.environ["DLLM_TRACE"]
    if "{rank}" in _p:
        _p = _p.replace("{rank}", os.environ.get("RANK", "0"))
    tracer.enable(_p)
    import atexit
    atexit.register(tracer.dump)

span = tracer.span
gpu_span = tracer.gpu_span
counter = tracer.counter
instant = tracer.instant
enable = tracer.enable
disable = tracer.disable
dump = tracer.dump
