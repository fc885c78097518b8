"""Power telemetry: amdsmi socket-power sampler (replaces the reference's jtop logger).

Reference: ``src/tests/logging_power.py`` (jtop @ 1 Hz, lines ``"%Y-%m-%d %H:%M:%S.%f: <mW>"``),
``src/tests/routing_chatbot_tester.py:199-254`` (log parsing; left-Riemann energy integration),
``src/tests/chatbot_tester.py:207-251`` (legacy: plain sum of 1 Hz samples).

Here a background thread samples every GPU's socket power through ``amdsmi`` (default 10 Hz) and
keeps samples in memory; it can also write the reference log format.  When amdsmi or a GPU is
unavailable the sampler records nothing and every energy reads 0.0 (reported as such).
"""
from __future__ import annotations

import os
import threading
import time
from datetime import datetime
from typing import Dict, List, Optional, Sequence, Tuple

TS_FMT = "%Y-%m-%d %H:%M:%S.%f"


class PowerSampler:
    def __init__(self, gpus: Optional[Sequence[int]] = None, hz: float = 10.0, log_path: Optional[str] = None):
        self.hz = hz
        self.log_path = log_path
        self.samples: Dict[int, List[Tuple[datetime, int]]] = {}
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._handles = []
        self.available = False
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            hs = amdsmi.amdsmi_get_processor_handles()
            idx = list(range(len(hs))) if gpus is None else [g for g in gpus if g < len(hs)]
            self._handles = [(i, hs[i]) for i in idx]
            self._amdsmi = amdsmi
            self.available = bool(self._handles)
        except Exception:
            self.available = False
        for i, _ in self._handles:
            self.samples[i] = []

    def read_mw(self, handle) -> int:
        info = self._amdsmi.amdsmi_get_power_info(handle)
        for key in ("current_socket_power", "average_socket_power", "socket_power"):
            v = info.get(key)
            if isinstance(v, (int, float)) and v > 0:
                return int(float(v) * 1000.0)  # W -> mW
        return 0

    def _loop(self) -> None:
        period = 1.0 / self.hz
        fh = open(self.log_path, "a") if self.log_path else None
        try:
            while not self._stop.is_set():
                t0 = time.time()
                now = datetime.now()
                for i, h in self._handles:
                    try:
                        mw = self.read_mw(h)
                    except Exception:
                        mw = 0
                    self.samples[i].append((now, mw))
                    if fh:
                        fh.write(f"{now.strftime(TS_FMT)}: {mw}\n")
                if fh:
                    fh.flush()
                self._stop.wait(max(0.0, period - (time.time() - t0)))
        finally:
            if fh:
                fh.close()

    def start(self) -> "PowerSampler":
        if self.available and self._thread is None:
            self._thread = threading.Thread(target=self._loop, daemon=True)
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None

    def energy_mj(self, gpus: Sequence[int], start: datetime, end: datetime) -> float:
        return sum(energy_for_window(dict(self.samples.get(g, [])), start, end) for g in gpus)


def parse_power_log(path: str) -> Dict[datetime, int]:
    """Parse ``"<timestamp>: <mW>"`` lines (reference log format); bad lines are skipped."""
    out: Dict[datetime, int] = {}
    if not os.path.exists(path):
        return out
    with open(path, "r") as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            ts_s, sep, p_s = line.rpartition(":")
            if not sep:
                continue
            ts = None
            for fmt in (TS_FMT, "%Y-%m-%d %H:%M:%S"):
                try:
                    ts = datetime.strptime(ts_s.strip(), fmt)
                    break
                except ValueError:
                    pass
            if ts is None:
                continue
            try:
                out[ts] = int(p_s.strip())
            except ValueError:
                continue
    return out


def energy_for_window(power: Dict[datetime, int], start: datetime, end: datetime) -> float:
    """Left-Riemann integral of mW samples inside [start, end] -> mJ (reference new harness)."""
    pts = sorted((t, p) for t, p in power.items() if start <= t <= end)
    e = 0.0
    for (t0, p0), (t1, _) in zip(pts, pts[1:]):
        dt = (t1 - t0).total_seconds()
        if dt > 0:
            e += p0 * dt
    return e


def energy_sum_1hz(power: Dict[datetime, int], start: datetime, end: datetime) -> float:
    """Legacy harness energy: plain sum of the samples in the window (1 Hz -> mJ)."""
    return float(sum(p for t, p in power.items() if start <= t <= end))
