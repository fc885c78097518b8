"""Local pool supervisor — replaces the reference's SSH ``ServerManager``
(src/models/server_manager.py:66-190: pexpect SSH bring-up, ``ssh -N -L`` tunnel, TCP-port
liveness, /health readiness, ``pkill -f`` teardown).

On one 8xMI355X node there is no SSH hop: each pool worker is a child process pinned to its GPU
subset with ``HIP_VISIBLE_DEVICES`` (tp > 1 pools are launched under torchrun with one rank per
GPU), reached over loopback HTTP.  The supervisor
  * starts workers and waits for ``/health`` (bounded),
  * stops them by PID / process group it owns (never by pattern),
  * restarts a worker whose process died (``ensure``/``watch``), counting restarts,
  * exposes ``is_running`` (process alive AND healthy).
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import sys
import threading
import time
import urllib.request
from dataclasses import dataclass, field
from typing import Dict, List, Optional


@dataclass
class PoolSpec:
    name: str
    port: int
    gpus: List[int] = field(default_factory=list)
    kind: str = "engine"
    model: str = "tinyllama-1.1b"
    max_new_tokens: int = 256
    temperature: float = 0.0
    tp: int = 1
    extra_args: List[str] = field(default_factory=list)

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}"


class Supervisor:
    def __init__(self, specs: List[PoolSpec], log_dir: str = "gpurun_out/pools", startup_timeout_s: float = 300.0):
        self.specs = {s.name: s for s in specs}
        self.procs: Dict[str, subprocess.Popen] = {}
        self.restarts: Dict[str, int] = {s.name: 0 for s in specs}
        self.log_dir = log_dir
        self.startup_timeout_s = startup_timeout_s
        self._lock = threading.Lock()
        self._watch: Optional[threading.Thread] = None
        self._stop = threading.Event()

    def _cmd(self, s: PoolSpec) -> List[str]:
        base = ["-m", "distributed_llm_amd.pools.worker", "--name", s.name, "--port", str(s.port), "--kind", s.kind,
                "--model", s.model, "--max-new-tokens", str(s.max_new_tokens), "--temperature", str(s.temperature),
                *s.extra_args]
        if s.tp > 1:
            # torchrun's -m runs the worker as a module in every rank (one rank per GPU of the pool)
            return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={s.tp}",
                    "--master-addr", "127.0.0.1", "--master-port", str(29600 + s.port % 1000), *base]
        return [sys.executable, *base]

    def healthy(self, name: str, timeout: float = 1.0) -> bool:
        try:
            with urllib.request.urlopen(self.specs[name].url + "/health", timeout=timeout) as r:
                return json.loads(r.read().decode()).get("ok") is True
        except Exception:
            return False

    def alive(self, name: str) -> bool:
        p = self.procs.get(name)
        return p is not None and p.poll() is None

    def is_running(self, name: str) -> bool:
        return self.alive(name) and self.healthy(name)

    def start(self, name: str, wait: bool = True) -> bool:
        with self._lock:
            if self.alive(name):
                return self.healthy(name) or (self._wait(name) if wait else True)
            s = self.specs[name]
            env = dict(os.environ)
            if s.gpus:
                env["HIP_VISIBLE_DEVICES"] = ",".join(map(str, s.gpus))
            env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
            os.makedirs(self.log_dir, exist_ok=True)
            log = open(os.path.join(self.log_dir, f"{name}.log"), "ab")
            self.procs[name] = subprocess.Popen(self._cmd(s), env=env, stdout=log, stderr=subprocess.STDOUT,
                                                start_new_session=True)
        return self._wait(name) if wait else True

    def _wait(self, name: str) -> bool:
        t0 = time.time()
        while time.time() - t0 < self.startup_timeout_s:
            if not self.alive(name):
                return False
            if self.healthy(name):
                return True
            time.sleep(0.25)
        return False

    def stop(self, name: str, timeout: float = 10.0) -> None:
        with self._lock:
            p = self.procs.pop(name, None)
        if p is None or p.poll() is not None:
            return
        try:
            os.killpg(p.pid, signal.SIGTERM)  # the group this supervisor created for the worker
            p.wait(timeout=timeout)
        except (ProcessLookupError, subprocess.TimeoutExpired):
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass

    def start_all(self) -> Dict[str, bool]:
        return {n: self.start(n) for n in self.specs}

    def stop_all(self) -> None:
        self._stop.set()
        for n in list(self.procs):
            self.stop(n)

    def ensure(self, name: str) -> bool:
        """Restart a dead worker (failure detection + elastic recovery)."""
        if self.alive(name):
            return True
        self.restarts[name] += 1
        return self.start(name)

    def watch(self, interval_s: float = 2.0) -> None:
        def loop():
            while not self._stop.wait(interval_s):
                for n in list(self.specs):
                    if n in self.procs and not self.alive(n):
                        self.ensure(n)
        self._watch = threading.Thread(target=loop, daemon=True)
        self._watch.start()
