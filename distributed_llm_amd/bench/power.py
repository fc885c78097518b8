"""Power telemetry: amdsmi socket-power sampler (replaces the reference's jtop logger).

Reference: ``src/tests/logging_power.py`` (jtop @ 1 Hz, lines ``"%Y-%m-%d %H:%M:%S.%f: <mW>"``),
``src/tests/routing_chatbot_tester.py:199-254`` (log parsing; left-Riemann energy integration),
``src/tests/chatbot_tester.py:207-251`` (legacy: plain sum of 1 Hz samples).

Here a background thread samples every GPU's socket power through ``amdsmi`` (default 10 Hz) and
keeps samples in memory; it can also write the reference log format.  When amdsmi or a GPU is
unavailable the sampler records nothing and every energy reads 0.0 (reported as such).

Per-query energy (the reference integrates power over each query window) is measured from the
GPU's cumulative energy counter (``amdsmi_get_energy_count``): ``mark()`` snapshots it at a query's
start and end and ``energy_between`` returns the delta, so a 100 ms query reads its real energy
instead of the 0 mJ a 1-10 Hz sample sum gives when no sample falls inside the window.  Where the
counter is unavailable the fallback is a trapezoid integral of the power trace linearly
interpolated at the window's boundaries (``energy_for_window_trapz``), which also covers windows
shorter than one sample period.  Energy is a property of a GPU, not of a tier: when tiers share a
GPU the per-query figure is that GPU's energy during the query (the harness is sequential, so
windows never overlap).
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

    def counter_mj(self, handle) -> Optional[float]:
        """The GPU's cumulative energy counter in mJ (None if the driver does not expose it)."""
        try:
            d = self._amdsmi.amdsmi_get_energy_count(handle)
            acc, res = d.get("energy_accumulator"), d.get("counter_resolution")
            if acc is None or not res:
                return None
            return float(acc) * float(res) / 1000.0   # counter units x uJ/unit -> mJ
        except Exception:
            return None

    def mark(self) -> "EnergyMark":
        """Snapshot (wall time, energy counter per GPU) at a query boundary."""
        cnt = {}
        for i, h in self._handles:
            cnt[i] = self.counter_mj(h)
        return EnergyMark(datetime.now(), cnt)

    def energy_between(self, gpus: Sequence[int], m0: "EnergyMark", m1: "EnergyMark") -> Tuple[float, str]:
        """Energy (mJ) of ``gpus`` between two marks and the method used: ``counter`` (energy
        counter delta), ``trapz`` (interpolated power trace) or ``none``."""
        total, method = 0.0, "none"
        for g in gpus:
            c0, c1 = m0.counters.get(g), m1.counters.get(g)
            if c0 is not None and c1 is not None and c1 >= c0:
                total += c1 - c0
                method = "counter"
                continue
            pts = self.samples.get(g, [])
            if pts:
                total += energy_for_window_trapz(pts, m0.time, m1.time)
                method = "trapz" if method == "none" else method
        return total, method

    def energy_mj(self, gpus: Sequence[int], start: datetime, end: datetime) -> float:
        """Energy of ``gpus`` over [start, end] from the sampled power trace (trapezoid over the
        trace interpolated at the window's boundaries)."""
        return sum(energy_for_window_trapz(self.samples.get(g, []), start, end) for g in gpus)


class BusySampler:
    """GPU busy share over a window: amdsmi's graphics-engine activity (%, the firmware's own
    utilisation counter) sampled by a thread at ``hz``.  Unlike a kernel trace it costs the host
    nothing measurable, so the step loop runs as in the timed bench.  ``stop()`` returns the mean
    (None when amdsmi or the counter is unavailable)."""

    def __init__(self, smi_idx: int, hz: float = 20.0):
        self.hz, self.vals = hz, []
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._h = None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self._smi = amdsmi
            self._h = amdsmi.amdsmi_get_processor_handles()[smi_idx]
            self._read()
        except Exception:
            self._h = None

    def _read(self) -> float:
        v = self._smi.amdsmi_get_gpu_activity(self._h).get("gfx_activity")
        return float(v)

    def _loop(self) -> None:
        period = 1.0 / self.hz
        while not self._stop.wait(period):
            try:
                self.vals.append(self._read())
            except Exception:
                pass

    def start(self) -> "BusySampler":
        if self._h is not None:
            self._thread = threading.Thread(target=self._loop, daemon=True, name="busy-sampler")
            self._thread.start()
        return self

    def stop(self) -> Optional[float]:
        if self._thread is None:
            return None
        self._stop.set()
        self._thread.join()
        return sum(self.vals) / len(self.vals) if self.vals else None


def smi_index_for_cuda(device: int) -> int:
    """amdsmi processor index of HIP device ``device`` (matched by PCI bus id: amdsmi lists every
    GPU the driver sees, HIP only the visible ones), falling back to the HIP index."""
    try:
        import amdsmi
        import torch
        props = torch.cuda.get_device_properties(device)
        want = (getattr(props, "pci_domain_id", 0), props.pci_bus_id, props.pci_device_id)
        amdsmi.amdsmi_init()
        for i, h in enumerate(amdsmi.amdsmi_get_processor_handles()):
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(h)          # "dddd:bb:dd.f"
            dom, bus, rest = bdf.split(":")
            if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
                return i
    except Exception:
        pass
    return device


class EnergyMark:
    """Wall time plus each GPU's energy counter (mJ, or None) at one instant."""
    __slots__ = ("time", "counters")

    def __init__(self, time_: datetime, counters: Dict[int, Optional[float]]):
        self.time = time_
        self.counters = counters


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


def energy_for_window_trapz(samples, start: datetime, end: datetime) -> float:
    """Integral (mJ) of a mW trace over [start, end]: the trace is linearly interpolated at both
    boundaries (held constant beyond its first / last sample) and integrated with the trapezoid
    rule, so the segments that straddle the window's edges count and a window shorter than one
    sample period still reads power x duration.  ``samples``: (time, mW) pairs or a dict."""
    pts = sorted(samples.items() if isinstance(samples, dict) else samples)
    if not pts or end <= start:
        return 0.0

    def at(t: datetime) -> float:
        if t <= pts[0][0]:
            return float(pts[0][1])
        if t >= pts[-1][0]:
            return float(pts[-1][1])
        lo, hi = 0, len(pts) - 1
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if pts[mid][0] <= t:
                lo = mid
            else:
                hi = mid
        (t0, p0), (t1, p1) = pts[lo], pts[hi]
        span = (t1 - t0).total_seconds()
        w = (t - t0).total_seconds() / span if span > 0 else 0.0
        return p0 + (p1 - p0) * w

    knots = [(start, at(start))] + [(t, float(p)) for t, p in pts if start < t < end] + [(end, at(end))]
    e = 0.0
    for (t0, p0), (t1, p1) in zip(knots, knots[1:]):
        e += 0.5 * (p0 + p1) * (t1 - t0).total_seconds()
    return e


def energy_sum_1hz(power: Dict[datetime, int], start: datetime, end: datetime) -> float:
    """Legacy harness energy: plain sum of the samples in the window (1 Hz -> mJ)."""
    return float(sum(p for t, p in power.items() if start <= t <= end))
