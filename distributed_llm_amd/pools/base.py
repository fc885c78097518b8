"""Pool clients — what the orchestrator dispatches to (reference L3 device clients).

Reference: ``src/models/nano.py:10-40``, ``src/models/orin.py:12-29`` (HTTP via SSH tunnel,
lazy server start), ``src/models/server_manager.py`` (SSH lifecycle) and the device shim
prompt format ``src/devices/nano_api.py:49-52`` (``"role: content"`` lines).

A pool is one model tier hosted on a set of GPUs of this node:
  * ``EnginePool``  — in-process ``engine.LLMEngine`` (this process owns the pool's GPUs);
  * ``HTTPPool``    — a pool-worker process (``pools.worker``) reached over loopback HTTP
                      with the reference ``/query`` protocol, and a request timeout on BOTH
                      tiers (the reference's Orin client has none, quirk 5);
  * ``EchoPool``    — deterministic CPU backend for the plumbing config (BASELINE config 1);
  * ``FaultInjectingPool`` — wraps any pool to drop / delay / fail requests (tests).
Every pool exposes ``process(history) -> {"response": ...} | {"error": ...}``,
optionally ``process_batch(histories)``, and a ``server_manager`` with the reference's
``start_server / stop_server / is_server_running`` names.
"""
from __future__ import annotations

import json
import random
import threading
import time
import urllib.error
import urllib.request
from typing import Any, Callable, Dict, List, Optional, Sequence

from ..config import LARGE, SMALL


def format_prompt(query: Any) -> str:
    """Reference device-shim formatting: ``"{role}: {content}"`` lines joined by newlines."""
    if isinstance(query, list):
        return "\n".join(f"{m.get('role', 'user')}: {m.get('content', '')}" for m in query).strip()
    return str(query).strip()


class Coalescer:
    """Merge concurrent submissions into one downstream batch call (leader/follower).

    ``fn(items) -> results`` is called with the items of every caller that arrived while the
    previous call was in flight, so N concurrent HTTP requests to a remote / tensor-parallel pool
    become one batched exchange instead of N serialised ones.  The caller that finds the pool
    idle drives; the others wait for their slice of the results.
    """

    def __init__(self, fn):
        self.fn = fn
        self._lock = threading.Lock()
        self._queue: List[Dict[str, Any]] = []
        self._busy = False
        self.calls = 0
        self.items = 0

    def submit(self, items: Sequence[Any]) -> List[Any]:
        job = {"items": list(items), "done": threading.Event(), "out": None, "err": None}
        with self._lock:
            self._queue.append(job)
            lead = not self._busy
            if lead:
                self._busy = True
        if lead:
            while True:
                with self._lock:
                    jobs, self._queue = self._queue, []
                    if not jobs:
                        self._busy = False
                        break
                flat = [it for j in jobs for it in j["items"]]
                try:
                    res = list(self.fn(flat))
                    if len(res) != len(flat):
                        raise RuntimeError(f"batch returned {len(res)} results for {len(flat)} items")
                    err = None
                except Exception as e:  # every waiter sees the failure
                    res, err = [None] * len(flat), e
                self.calls += 1
                self.items += len(flat)
                k = 0
                for j in jobs:
                    n = len(j["items"])
                    j["out"], j["err"] = res[k:k + n], err
                    k += n
                    j["done"].set()
        job["done"].wait()
        if job["err"] is not None:
            raise job["err"]
        return job["out"]


class PoolHandle:
    """One request submitted without waiting (``submit_batch``): ``done`` fires when ``reply`` (a
    pool payload: ``{"response": ...}`` or ``{"error": ...}``) is set, and ``notify(handle)`` (an
    event-driven client's completion queue) is called exactly once, from whichever thread
    completed it.  Remote pools complete handles from their receiver thread; a deadline reaper
    fails handles a hung pool never answers (the reference's per-request ``timeout=(5, 180)``)."""

    __slots__ = ("done", "reply", "notify", "deadline", "rp", "_lock")

    def __init__(self, notify: Optional[Callable[["PoolHandle"], None]] = None, deadline: Optional[float] = None):
        self.done = threading.Event()
        self.reply: Optional[Dict[str, Any]] = None
        self.notify = notify
        self.deadline = deadline
        self.rp = None               # ReplicatedPool bookkeeping: {id(pool): [replica, released]}
        self._lock = threading.Lock()

    def complete(self, reply: Dict[str, Any]) -> bool:
        """Set the reply once (later completions - a late reply after a timeout - are dropped)."""
        with self._lock:
            if self.done.is_set():
                return False
            self.reply = reply
            self.done.set()
        if self.notify is not None:
            try:
                self.notify(self)
            except Exception:  # noqa: BLE001 - a client sink must never kill a pool thread
                pass
        return True

    def payload(self) -> Dict[str, Any]:
        return self.reply if self.reply is not None else {"error": "request not finished"}


class ThreadSubmit:
    """``submit_batch`` / ``collect`` for a pool whose only entry is the blocking
    ``process_batch`` (echo / fault-injecting / HTTP pools): the batch is served on a small
    executor and its handles complete when it returns, so an event-driven client is never blocked
    by a synchronous pool."""

    _submit_workers = 8

    def submit_batch(self, histories, overrides: Optional[Dict[str, Any]] = None, notify=None) -> List[PoolHandle]:
        ex = getattr(self, "_submit_ex", None)
        if ex is None:
            from concurrent.futures import ThreadPoolExecutor
            ex = self._submit_ex = ThreadPoolExecutor(self._submit_workers, thread_name_prefix=f"dllm-sub-{self.name}")
        hs = [PoolHandle(notify) for _ in histories]

        def run():
            try:
                res = list(self.process_batch(list(histories)))
                if len(res) != len(hs):
                    raise RuntimeError(f"pool returned {len(res)} results for {len(hs)} requests")
            except Exception as e:  # noqa: BLE001 - every handle sees the failure
                res = [{"error": f"pool {self.name} failed: {e}"}] * len(hs)
            for h, r in zip(hs, res):
                h.complete(r)
        ex.submit(run)
        return hs

    @staticmethod
    def collect(handles) -> List[Dict[str, Any]]:
        return [h.payload() for h in handles]


class NullServerManager:
    """In-process pools are always 'running'; kept for harness API compatibility."""

    def __init__(self):
        self.running = True

    def start_server(self):
        self.running = True

    def stop_server(self):
        self.running = True  # in-process pools stay resident (weights stay in HBM)

    def is_server_running(self) -> bool:
        return self.running


class PoolClient:
    name: str = SMALL

    def __init__(self):
        self.server_manager = NullServerManager()

    def process(self, history: Any) -> Dict[str, Any]:
        raise NotImplementedError

    def process_batch(self, histories: Sequence[Any]) -> List[Dict[str, Any]]:
        return [self.process(h) for h in histories]

    def health(self) -> Dict[str, Any]:
        return {"ok": True}


class EchoPool(ThreadSubmit, PoolClient):
    """Deterministic CPU backend: echoes the last user turn, ``tokens_per_reply`` words long."""

    def __init__(self, name: str = SMALL, tokens_per_reply: int = 16, delay_s: float = 0.0):
        super().__init__()
        self.name = name
        self.tokens_per_reply = tokens_per_reply
        self.delay_s = delay_s
        self.calls = 0
        self._lock = threading.Lock()

    def process(self, history: Any) -> Dict[str, Any]:
        prompt = format_prompt(history)
        if not prompt:
            return {"error": "No query provided"}
        with self._lock:
            self.calls += 1
        if self.delay_s:
            time.sleep(self.delay_s)
        last = prompt.rsplit("\n", 1)[-1]
        words = (f"[{self.name}] " + last).split()
        reply = " ".join((words * (self.tokens_per_reply // max(len(words), 1) + 1))[:self.tokens_per_reply])
        return {"response": reply, "num_tokens": self.tokens_per_reply}


class FaultInjectingPool(ThreadSubmit, PoolClient):
    """Wraps a pool; ``mode`` in {"ok", "error", "timeout", "flaky"}."""

    def __init__(self, inner: PoolClient, mode: str = "error", p: float = 0.5, seed: int = 0,
                 timeout_s: float = 0.0):
        super().__init__()
        self.inner, self.mode, self.p, self.timeout_s = inner, mode, p, timeout_s
        self.name = inner.name
        self.server_manager = inner.server_manager
        self._rng = random.Random(seed)

    def process(self, history: Any) -> Dict[str, Any]:
        if self.mode == "error" or (self.mode == "flaky" and self._rng.random() < self.p):
            return {"error": f"injected fault on {self.name}"}
        if self.mode == "timeout":
            time.sleep(self.timeout_s)
            return {"error": f"Request timed out on {self.name}"}
        return self.inner.process(history)

    def process_batch(self, histories):
        return [self.process(h) for h in histories]


class HTTPServerManager:
    """Liveness/readiness of a pool-worker process (local; no SSH on one node)."""

    def __init__(self, url: str, supervisor=None, pool_name: str = SMALL):
        self.url = url.rstrip("/")
        self.supervisor = supervisor
        self.pool_name = pool_name

    def is_server_running(self) -> bool:
        try:
            with urllib.request.urlopen(self.url + "/health", timeout=1.0) as r:
                return json.loads(r.read().decode()).get("ok", False) is True
        except Exception:
            return False

    def start_server(self):
        if self.supervisor is not None and not self.is_server_running():
            if self.pool_name in self.supervisor.procs:
                self.supervisor.ensure(self.pool_name)   # died: restart, counted
            self.supervisor.start(self.pool_name)

    def stop_server(self):
        if self.supervisor is not None:
            self.supervisor.stop(self.pool_name)


class HTTPPool(PoolClient):
    def __init__(self, name: str, url: str, timeout_s: float = 180.0, connect_timeout_s: float = 5.0,
                 supervisor=None, options: Optional[Dict[str, Any]] = None):
        super().__init__()
        self.name = name
        self.url = url.rstrip("/")
        self.timeout_s = timeout_s
        self.options = dict(options or {})
        self.server_manager = HTTPServerManager(url, supervisor, name)

    def _post(self, payload: Dict[str, Any]) -> Dict[str, Any]:
        req = urllib.request.Request(self.url + "/query", data=json.dumps(payload).encode(),
                                     headers={"Content-Type": "application/json"}, method="POST")
        try:
            with urllib.request.urlopen(req, timeout=self.timeout_s) as r:
                ct = (r.headers.get("Content-Type") or "").lower()
                body = r.read().decode("utf-8", "replace")
                if "application/json" not in ct:
                    return {"error": f"Non-JSON response ({r.status})", "body": body[:500]}
                return json.loads(body) if body else {"error": "Empty response"}
        except urllib.error.HTTPError as e:
            try:
                return json.loads(e.read().decode())
            except Exception:
                return {"error": f"HTTP {e.code}"}
        except TimeoutError:
            return {"error": f"Request timed out on {self.name}"}
        except Exception as e:
            return {"error": f"Request failed: {e}"}

    def process(self, history: Any) -> Dict[str, Any]:
        if not self.server_manager.is_server_running():
            self.server_manager.start_server()
        return self._post({"query": history, **self.options})

    def process_batch(self, histories):
        if not self.server_manager.is_server_running():
            self.server_manager.start_server()
        res = self._post({"queries": list(histories), **self.options})
        if isinstance(res, dict) and "responses" in res:
            return res["responses"]
        return [res] * len(histories)

    def health(self) -> Dict[str, Any]:
        return {"ok": self.server_manager.is_server_running()}


class EnginePool(PoolClient):
    """A pool served by an in-process ``engine.LLMEngine``."""

    # Generation prompt appended after the reference's "role: content" lines (a minimal chat
    # template): the reply then continues the prompt text exactly, so the next turn's prompt
    # extends prompt + reply and the engine's session memo / prefix cache reuse the whole turn.
    GENERATION_PROMPT = "\nassistant: "

    def __init__(self, name: str, engine, max_new_tokens: int = 256, temperature: float = 0.0,
                 top_k: int = 0, top_p: float = 1.0, generation_prompt: Optional[str] = None):
        super().__init__()
        self.name = name
        self.generation_prompt = self.GENERATION_PROMPT if generation_prompt is None else generation_prompt
        self.engine = engine
        self.max_new_tokens = max_new_tokens
        self.temperature = temperature
        self.top_k = top_k
        self.top_p = top_p

    def prompt_for(self, history: Any) -> str:
        return format_prompt(history) + self.generation_prompt

    def _params(self, overrides: Optional[Dict[str, Any]] = None):
        from ..engine.sampling import SamplingParams
        o = overrides or {}
        n = int(o.get("num_predict", self.max_new_tokens))
        return SamplingParams(max_new_tokens=self.max_new_tokens if n < 0 else n,
                              temperature=float(o.get("temperature", self.temperature)),
                              top_k=int(o.get("top_k", self.top_k)),
                              top_p=float(o.get("top_p", self.top_p)))

    def process(self, history: Any, overrides: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        return self.process_batch([history], overrides)[0]

    def process_batch(self, histories, overrides: Optional[Dict[str, Any]] = None):
        prompts = [self.prompt_for(h) for h in histories]
        return self.to_payloads(self.engine.generate(prompts, self._params(overrides)))

    def submit_batch(self, histories, overrides: Optional[Dict[str, Any]] = None, notify=None):
        """Non-blocking ``process_batch`` (the engine's background loop must run): request handles
        whose ``done`` event fires on completion (and which are passed to ``notify``, if given);
        ``collect`` turns finished handles into payloads."""
        return self.engine.submit([self.prompt_for(h) for h in histories], self._params(overrides), notify=notify)

    def collect(self, handles) -> List[Dict[str, Any]]:
        return self.to_payloads(self.engine.results(handles))

    @staticmethod
    def to_payloads(outs) -> List[Dict[str, Any]]:
        res = []
        for o in outs:
            if o.error:
                res.append({"error": o.error})
            else:
                res.append({"response": o.text, "num_tokens": o.num_generated,
                            "latency_ms": o.latency_ms,
                            "timing": {"queue_ms": o.queue_ms, "ttft_ms": o.ttft_ms,
                                       "prefill_tokens": o.num_prefill, "cached_tokens": o.num_cached,
                                       "decode_tok_s": o.decode_tok_s}})
        return res

    def health(self) -> Dict[str, Any]:
        return {"ok": True, **self.engine.stats()}


def default_pools(config: Dict[str, Any]) -> Dict[str, PoolClient]:
    """Pools from ``config["pools"]`` or echo pools (plumbing config) when none given."""
    spec = config.get("pools")
    if not spec:
        return {SMALL: EchoPool(SMALL), LARGE: EchoPool(LARGE, tokens_per_reply=48)}
    from .factory import build_pools
    return build_pools(spec)
