"""Pools that live on other ranks of the node, and data-parallel replica sets.

The reference reaches a device with one blocking HTTP request per turn through an SSH tunnel,
bounded by ``timeout=(5, 180)`` and failing over on any error (src/models/nano.py:23-38,
src/router.py:277-282); liveness is a TCP connect and readiness a ``/health`` poll
(src/models/server_manager.py:52-61,123-131).  Here a pool is a process group on this node:

* **control plane** — JSON messages on a 2-rank CPU (gloo) group per remote pool leader.  Every
  request carries an id; any number are in flight at once; replies come back out of order and a
  receiver thread hands each to its waiting caller.  A caller waits at most ``timeout_s`` and
  then gets an error payload (the orchestrator fails over); a pool process that dies closes its
  sockets, which fails every in-flight request at once.  The router never blocks on a dead or
  hung pool.
* **data plane** — the router<->leader pair group (gloo by default, RCCL with
  ``DLLM_DATA_PLANE=rccl``): prompt token ids for a failover hand-off (``process_failover``: the
  router tokenises with the target pool's tokenizer and ships int32 ids, so the surviving pool
  prefills ids directly) and the periodic 4 KiB data-plane ping.  Every transfer and the lock
  that orders them have deadlines (``data_timeout_s``); a data-plane failure retires the data
  plane of that pool (the hand-off falls back to the text prompt on the control plane) instead
  of blocking a caller.
* **health** — a probe thread pings every ``probe_interval_s`` on the control plane (answered by
  the leader's receiver thread immediately, never queued behind generation) and every
  ``data_probe_every``-th time on the data plane; two consecutive control-plane failures mark
  the pool dead; every probe result is reported to ``on_health`` (the orchestrator feeds the
  perf router).  Recovery: a pool marked dead by probes while its transport is intact (a hung
  engine, a long GC pause) is probed on, and ``revive_after`` consecutive good probes put it back
  in service — the reference's lazy restart-on-next-call (src/models/nano.py:19-21) for a pool
  that cannot be respawned inside one torch.distributed job; a pool whose process died (transport
  closed) stays out (restartable pools are the supervised HTTP workers, pools.supervisor).
* **pool side** (``PoolLeader``) — the receiver thread answers pings inline and hands each
  generate request to a worker thread that calls ``engine.generate``; data-plane operations
  (token receives, data pings) run in order on a dedicated data thread with deadlines, so a
  router that dies mid-transfer never wedges the receiver loop; the engine runs its background
  step loop, so concurrent requests from the router JOIN ONE continuous batch.
  Tensor-parallel pools keep their members in lockstep with the engine's mirror channel
  (``LLMEngine.enable_tp_mirror``), not per request.
* ``ReplicatedPool`` — several replicas of one tier (data parallel), least-loaded dispatch.
"""
from __future__ import annotations

import itertools
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Callable, Dict, List, Optional, Sequence

from ..parallel import p2p
from ..utils.faults import fault
from .base import EnginePool, NullServerManager, PoolClient, PoolHandle, format_prompt

TAG_REQ, TAG_REP = 1, 2


class RemoteServerManager(NullServerManager):
    def __init__(self, pool: "RemotePool"):
        super().__init__()
        self.pool = pool

    def is_server_running(self) -> bool:
        return self.pool.alive


class _Pending:
    __slots__ = ("event", "reply")

    def __init__(self):
        self.event = threading.Event()
        self.reply: Optional[Dict[str, Any]] = None


class RemotePool(PoolClient):
    def __init__(self, name: str, leader: int, ctrl_group, data_group=None, max_new_tokens: int = 256,
                 temperature: float = 0.0, top_k: int = 0, top_p: float = 1.0,
                 generation_prompt: str = EnginePool.GENERATION_PROMPT, timeout_s: float = 180.0,
                 tokenizer=None, on_health: Optional[Callable[[str, bool, Optional[float]], None]] = None,
                 data_timeout_s: float = 10.0, revive_after: int = 3):
        super().__init__()
        self.name = name
        self.leader = leader
        self.ctrl = ctrl_group
        self.data = data_group
        self.params = {"max_new_tokens": max_new_tokens, "temperature": temperature, "top_k": top_k, "top_p": top_p}
        self.generation_prompt = generation_prompt
        self.timeout_s = timeout_s
        self.tokenizer = tokenizer          # the pool's tokenizer (token-id hand-off), optional
        self.on_health = on_health
        self.alive = True
        self.transport_ok = True            # False once the control-plane receiver has died
        self.data_timeout_s = data_timeout_s
        self.data_error: Optional[str] = None   # set when the data plane was retired
        self.revive_after = revive_after
        self._good_probes = 0
        self.revivals = 0
        self.server_manager = RemoteServerManager(self)
        self._send_lock = threading.Lock()
        self._data_lock = threading.Lock()
        self._pending: Dict[int, _Pending] = {}
        self._plock = threading.Lock()
        self._ids = itertools.count(1)
        self.last_rtt_us: Optional[float] = None
        self.last_data_rtt_us: Optional[float] = None
        self.last_stats: Dict[str, Any] = {}
        self.timeouts = 0
        self.probe_failures = 0
        self._probe_stop = threading.Event()
        self._probe: Optional[threading.Thread] = None
        self._rx = threading.Thread(target=self._rx_loop, name=f"dllm-rx-{name}", daemon=True)
        self._rx.start()

    # ------------------------------------------------------------------ transport
    def prompt_for(self, history: Any) -> str:
        return format_prompt(history) + self.generation_prompt

    def _rx_loop(self) -> None:
        while True:
            try:
                msg = p2p.recv_obj(self.leader, self.ctrl, tag=TAG_REP)
            except Exception as e:  # peer died / transport closed: fail everything in flight
                self.transport_ok = False
                self._fail_all(f"pool {self.name} transport failed: {e}")
                return
            if msg.get("op") == "bye":
                self.transport_ok = False
                self._fail_all(f"pool {self.name} stopped")
                return
            with self._plock:
                ent = self._pending.pop(msg.get("id"), None)
            if isinstance(ent, PoolHandle):       # a submitted request: its own payload
                ent.complete(msg.get("result") or {"error": msg.get("error", "empty reply")})
            elif ent is not None:
                ent.reply = msg
                ent.event.set()

    def _fail_all(self, why: str) -> None:
        self.alive = False
        with self._plock:
            pend, self._pending = self._pending, {}
        for ent in pend.values():
            if isinstance(ent, PoolHandle):
                ent.complete({"error": why})
            else:
                ent.reply = {"error": why}
                ent.event.set()

    # bound on one control-plane send: a gloo send to a leader that died mid-conversation can block
    # instead of raising (seen in the config-4 leader-death rehearsal: the router's dispatch thread
    # hung in the send while the receiver thread had already seen the connection close)
    CTRL_SEND_TIMEOUT_S = 30.0

    def _send(self, msg: Dict[str, Any]) -> None:
        if not self.transport_ok:   # the receiver saw the connection close: never touch the pair again
            raise RuntimeError(f"pool {self.name} transport closed")
        with self._send_lock:
            try:
                p2p.send_obj(msg, self.leader, self.ctrl, tag=TAG_REQ, timeout_s=self.CTRL_SEND_TIMEOUT_S)
            except p2p.DataPlaneTimeout as e:   # a control-plane failure, not a data-plane one
                self.transport_ok = False
                raise RuntimeError(f"pool {self.name} control send: {e}") from e

    def data_ok(self) -> bool:
        return self.data is not None and self.data_error is None and self.alive

    def _retire_data(self, why: str) -> None:
        """Stop using the data plane of this pool (a pending transfer may still be posted on it)."""
        if self.data_error is None:
            self.data_error = why

    def _call(self, msg: Dict[str, Any], timeout: Optional[float] = None, data_fn=None,
              probe: bool = False) -> Dict[str, Any]:
        """Send one tagged request and wait for its reply at most ``timeout`` seconds."""
        if not self.alive and not (probe and self.transport_ok):
            return {"error": f"pool {self.name} unavailable"}
        rid = next(self._ids)
        msg["id"] = rid
        ent = _Pending()
        with self._plock:
            self._pending[rid] = ent
        try:
            if data_fn is None:
                self._send(msg)
            else:  # control message + its data-plane payload, in order w.r.t. other data ops
                if not self._data_lock.acquire(timeout=self.data_timeout_s):
                    raise p2p.DataPlaneTimeout("data plane busy (a transfer is stuck)")
                try:
                    self._send(msg)
                    data_fn()
                finally:
                    self._data_lock.release()
        except p2p.DataPlaneTimeout as e:
            with self._plock:
                self._pending.pop(rid, None)
            self._retire_data(str(e))
            return {"error": f"pool {self.name} data plane: {e}", "data_plane_failed": True}
        except Exception as e:
            with self._plock:
                self._pending.pop(rid, None)
            self._fail_all(f"pool {self.name} send failed: {e}")
            return {"error": f"pool {self.name} send failed: {e}"}
        if not ent.event.wait(self.timeout_s if timeout is None else timeout):
            with self._plock:
                self._pending.pop(rid, None)
            self.timeouts += 1
            return {"error": f"Request timed out on {self.name} after {timeout or self.timeout_s:.1f}s"}
        return ent.reply or {"error": "empty reply"}

    # ------------------------------------------------------------------ requests
    def process(self, history: Any) -> Dict[str, Any]:
        return self.process_batch([history])[0]

    def process_batch(self, histories: Sequence[Any], overrides: Optional[Dict[str, Any]] = None):
        params = dict(self.params, **(overrides or {}))
        rep = self._call({"op": "generate", "prompts": [self.prompt_for(h) for h in histories], "params": params})
        return self._results(rep, len(histories))

    def process_ids(self, prompt_ids: Sequence[Sequence[int]], overrides: Optional[Dict[str, Any]] = None):
        """Generate from prompt token ids shipped over the data plane (int32 tensors)."""
        params = dict(self.params, **(overrides or {}))
        ids = [list(map(int, p)) for p in prompt_ids]

        def ship():
            for p in ids:
                p2p.send_tokens(p, self.leader, self.data, timeout_s=self.data_timeout_s)
        rep = self._call({"op": "generate_ids", "n": len(ids), "params": params}, data_fn=ship)
        return self._results(rep, len(ids))

    def process_failover(self, history: Any) -> Dict[str, Any]:
        """Failover entry (orchestrator): hand the prompt over as token ids when this router has
        the pool's tokenizer and a live data plane, else (or if the hand-off fails on the data
        plane) as text on the control plane."""
        if self.tokenizer is not None and self.data_ok():
            r = self.process_ids([self.tokenizer.encode(self.prompt_for(history))])[0]
            if not (isinstance(r, dict) and "data plane" in str(r.get("error", ""))):
                return r
        return self.process(history)

    # ------------------------------------------------------------------ non-blocking requests
    def submit_batch(self, histories: Sequence[Any], overrides: Optional[Dict[str, Any]] = None,
                     notify=None) -> List[PoolHandle]:
        """Send the requests WITHOUT waiting: one tagged id per request, so the leader's engine
        admits each into its running continuous batch and answers each on its own as soon as it
        is done (``notify(handle)`` from the receiver thread).  Same deadline as ``process``: a
        request the pool never answers is failed by the reaper; a dead pool fails every handle.
        A pool already out of service returns handles that are done (error) and not notified."""
        params = dict(self.params, **(overrides or {}))
        return self._submit({"op": "submit", "prompts": [self.prompt_for(h) for h in histories], "params": params},
                            len(histories), notify)

    def submit_failover(self, histories: Sequence[Any], notify=None) -> List[PoolHandle]:
        """Non-blocking failover hand-off: the prompts go over the data plane as token ids (as
        ``process_failover``) when this router holds the pool's tokenizer and a live data plane,
        else as text on the control plane."""
        if self.tokenizer is not None and self.data_ok():
            ids = [list(map(int, self.tokenizer.encode(self.prompt_for(h)))) for h in histories]

            def ship():
                for p in ids:
                    p2p.send_tokens(p, self.leader, self.data, timeout_s=self.data_timeout_s)
            hs = self._submit({"op": "submit_ids", "n": len(ids), "params": dict(self.params)}, len(ids), notify,
                              data_fn=ship)
            if not any(h.done.is_set() and "data plane" in str(h.payload().get("error", "")) for h in hs):
                return hs
        return self.submit_batch(histories, notify=notify)

    def _submit(self, msg: Dict[str, Any], n: int, notify, data_fn=None) -> List[PoolHandle]:
        deadline = time.monotonic() + self.timeout_s
        hs = [PoolHandle(notify, deadline) for _ in range(n)]
        if not self.alive:
            for h in hs:
                h.reply = {"error": f"pool {self.name} unavailable"}
                h.done.set()
            return hs
        ids = [next(self._ids) for _ in range(n)]
        msg["ids"] = ids
        msg["id"] = 0
        with self._plock:
            for rid, h in zip(ids, hs):
                self._pending[rid] = h
        err = None
        try:
            if data_fn is None:
                self._send(msg)
            else:
                if not self._data_lock.acquire(timeout=self.data_timeout_s):
                    raise p2p.DataPlaneTimeout("data plane busy (a transfer is stuck)")
                try:
                    self._send(msg)
                    data_fn()
                finally:
                    self._data_lock.release()
        except p2p.DataPlaneTimeout as e:
            self._retire_data(str(e))
            err = {"error": f"pool {self.name} data plane: {e}", "data_plane_failed": True}
        except Exception as e:  # noqa: BLE001 - transport gone: this pool is out of service
            self._fail_all(f"pool {self.name} send failed: {e}")
            return hs
        if err is not None:
            with self._plock:
                for rid in ids:
                    self._pending.pop(rid, None)
            for h in hs:   # not sent / not shipped: done, not notified (the caller sees it at once)
                h.reply = err
                h.done.set()
            return hs
        self._start_reaper()
        return hs

    def _start_reaper(self) -> None:
        if getattr(self, "_reaper", None) is not None:
            return
        self._reaper = threading.Thread(target=self._reap_loop, name=f"dllm-reap-{self.name}", daemon=True)
        self._reaper.start()

    def _reap_loop(self, period_s: float = 0.5) -> None:
        """Fail submitted requests past their deadline (a hung pool): the caller fails over."""
        while not self._probe_stop.wait(period_s):
            now = time.monotonic()
            with self._plock:
                late = [rid for rid, e in self._pending.items()
                        if isinstance(e, PoolHandle) and e.deadline is not None and e.deadline < now]
                ents = [self._pending.pop(rid) for rid in late]
            for e in ents:
                self.timeouts += 1
                e.complete({"error": f"Request timed out on {self.name} after {self.timeout_s:.1f}s"})

    @staticmethod
    def collect(handles: Sequence[PoolHandle]) -> List[Dict[str, Any]]:
        return [h.payload() for h in handles]

    @staticmethod
    def _results(rep: Dict[str, Any], n: int) -> List[Dict[str, Any]]:
        res = rep.get("results")
        if not res or len(res) != n:
            return [{"error": rep.get("error", "empty reply")}] * n
        return res

    # ------------------------------------------------------------------ health
    def probe(self, timeout: float = 5.0) -> Dict[str, Any]:
        """Control-plane round trip + the pool's engine statistics (never queued behind work).
        Also sent to a pool marked dead while its transport is intact (revival)."""
        t0 = time.perf_counter()
        rep = self._call({"op": "ping"}, timeout=timeout, probe=True)
        if "error" in rep:
            return {"ok": False, "error": rep["error"]}
        self.last_rtt_us = (time.perf_counter() - t0) * 1e6
        self.last_stats = rep.get("stats", {})
        return {"ok": True, "rtt_us": self.last_rtt_us, **self.last_stats}

    def probe_data(self, timeout: float = 5.0) -> Dict[str, Any]:
        """4 KiB ping-pong on the data plane.  Every wait (the ordering lock, each transfer) is
        bounded by ``timeout``.  A failed TRANSFER retires the data plane (failover then ships
        text); a busy plane (a multi-prompt hand-off holds the ordering lock for up to n x its
        transfer deadline) only skips this probe."""
        if not self.data_ok():
            return {"ok": False, "error": self.data_error or "no data plane"}
        if not self._data_lock.acquire(timeout=timeout):
            return {"ok": True, "skipped": "data plane busy with a hand-off"}
        try:
            self._send({"op": "ping_data", "id": 0, "timeout_s": timeout})
            rtt = p2p.ping(self.leader, self.data, initiator=True, timeout_s=timeout)
        except Exception as e:  # noqa: BLE001 - DataPlaneTimeout or transport error
            self._retire_data(f"data-plane ping failed: {e}")
            return {"ok": False, "error": self.data_error}
        finally:
            self._data_lock.release()
        self.last_data_rtt_us = rtt
        return {"ok": True, "rtt_us": rtt}

    def start_probes(self, interval_s: float = 2.0, timeout_s: float = 5.0, data_probe_every: int = 5) -> None:
        """Periodic health probes on their own thread; two consecutive failures mark the pool dead."""
        if self._probe is not None:
            return

        def loop():
            k = 0
            while not self._probe_stop.wait(interval_s):
                if not self.alive and not self.transport_ok:
                    self._report(False, None)   # the pool process is gone: stays out of service
                    continue
                k += 1
                r = self.probe(timeout_s)
                if not self.alive:
                    # dead by probes, transport intact: revive after enough consecutive good probes
                    self._good_probes = self._good_probes + 1 if r["ok"] else 0
                    if self._good_probes >= self.revive_after:
                        self.alive, self.probe_failures, self._good_probes = True, 0, 0
                        self.revivals += 1
                        self._report(True, r.get("rtt_us"))
                    else:
                        self._report(False, None)
                    continue
                if r["ok"] and data_probe_every and k % data_probe_every == 0 and self.data_ok():
                    # a data-plane failure retires the data plane; the pool stays in service
                    self.probe_data(timeout_s)
                if r["ok"]:
                    self.probe_failures = 0
                    self._report(True, r.get("rtt_us"))
                else:
                    self.probe_failures += 1
                    if self.probe_failures >= 2:
                        self._fail_all(f"pool {self.name} failed {self.probe_failures} health probes: {r['error']}")
                    self._report(False, None)
        self._probe = threading.Thread(target=loop, name=f"dllm-probe-{self.name}", daemon=True)
        self._probe.start()

    def _report(self, ok: bool, rtt_us: Optional[float]) -> None:
        if self.on_health is not None:
            try:
                self.on_health(self.name, ok, rtt_us)
            except Exception:  # noqa: BLE001 - a health sink must never kill the probe thread
                pass

    def health(self) -> Dict[str, Any]:
        return self.probe()

    # ------------------------------------------------------------------ lifecycle
    def sync(self) -> None:
        """Barrier hand-off (bench timing): the leader barriers with its members and the node.  A
        leader that died (e.g. in the warmup) fails its pool here instead of raising in the router:
        the node barrier that follows then marks the node degraded."""
        try:
            self._send({"op": "sync", "id": 0})
        except Exception as e:  # noqa: BLE001 - transport gone
            self._fail_all(f"pool {self.name} sync failed: {e}")

    def stop(self) -> None:
        self._probe_stop.set()
        if self.alive:
            try:
                self._send({"op": "stop", "id": 0})
            except Exception:  # noqa: BLE001
                pass
            self._rx.join(timeout=30)
        self.alive = False


class PoolLeader:
    """Pool-side server of one pool leader rank (see module docstring)."""

    def __init__(self, engine, ctrl_group, data_group=None, router_rank: int = 0, on_sync=None,
                 max_workers: int = 64, data_timeout_s: float = 10.0):
        import queue
        self.engine = engine
        self.ctrl = ctrl_group
        self.data = data_group
        self.router = router_rank
        self.on_sync = on_sync
        self.data_timeout_s = data_timeout_s
        self.data_error: Optional[str] = None
        self._send_lock = threading.Lock()
        self._ex = ThreadPoolExecutor(max_workers=max_workers, thread_name_prefix="dllm-pool")
        # data-plane operations, in arrival order, off the receiver loop (bounded waits)
        self._dq: "queue.Queue" = queue.Queue()
        self._dthread = threading.Thread(target=self._data_loop, name="dllm-pool-data", daemon=True)
        self._dthread.start()
        # submitted requests (op "submit" / "submit_ids"): the engine's completion callback only
        # queues the finished sequence; this thread forms its payload and replies, so the engine's
        # step loop never blocks on the control-plane socket
        self._rq: "queue.Queue" = queue.Queue()
        # submits run on their own thread, in arrival order (tokenising a batch never delays the
        # receiver loop's answers to health pings)
        self._sub_ex = ThreadPoolExecutor(max_workers=1, thread_name_prefix="dllm-pool-submit")
        self._rthread = threading.Thread(target=self._reply_loop, name="dllm-pool-reply", daemon=True)
        self._rthread.start()

    def _data_loop(self) -> None:
        while True:
            msg = self._dq.get()
            if msg is None:
                return
            op = msg.get("op")
            if self.data_error is not None:   # retired: answer what needs an answer, move nothing
                if op == "generate_ids":
                    self._safe_reply({"id": msg["id"], "error": f"data plane retired: {self.data_error}"})
                elif op == "submit_ids":
                    for rid in msg["ids"]:
                        self._safe_reply({"id": rid, "error": f"data plane retired: {self.data_error}"})
                continue
            try:
                if op == "ping_data" and fault("die_on_data_ping") == "1":
                    os._exit(17)   # fault injection (tests): the leader dies during a data-plane ping
                if op == "ping_data":
                    p2p.ping(self.router, self.data, initiator=False,
                             timeout_s=float(msg.get("timeout_s") or self.data_timeout_s))
                elif op in ("generate_ids", "submit_ids"):
                    prompts = [p2p.recv_tokens(self.router, self.data, timeout_s=self.data_timeout_s).tolist()
                               for _ in range(int(msg["n"]))]
                    if op == "submit_ids":
                        self._submit(msg["ids"], prompts, msg.get("params"))
                    else:
                        self._ex.submit(self._generate, msg["id"], prompts, msg.get("params"))
            except Exception as e:  # noqa: BLE001 - DataPlaneTimeout / transport: retire, report
                self.data_error = str(e)
                if op == "generate_ids":
                    self._safe_reply({"id": msg["id"], "error": f"data plane: {e}"})
                elif op == "submit_ids":
                    for rid in msg["ids"]:
                        self._safe_reply({"id": rid, "error": f"data plane: {e}"})

    def _safe_reply(self, msg: Dict[str, Any]) -> None:
        try:
            self._reply(msg)
        except Exception:  # noqa: BLE001 - router gone
            pass

    def _reply(self, msg: Dict[str, Any]) -> None:
        with self._send_lock:
            p2p.send_obj(msg, self.router, self.ctrl, tag=TAG_REP)

    def _generate(self, rid: int, prompts, params) -> None:
        import os
        from ..engine.sampling import SamplingParams
        hang = fault("hang_on")
        if hang and any(isinstance(p, str) and hang in p for p in prompts):
            time.sleep(fault("hang_s", 5.0, float))   # fault injection (tests)
        try:
            sp = SamplingParams.from_dict(params or {})
            outs = self.engine.generate(prompts, sp)
            rep = {"id": rid, "results": EnginePool.to_payloads(outs)}
        except Exception as e:  # report, never kill the pool loop
            rep = {"id": rid, "error": f"engine failed: {e}"}
        try:
            self._reply(rep)
        except Exception:  # noqa: BLE001 - router gone; nothing to report to
            pass

    def _submit(self, rids, prompts, params) -> None:
        """Admit requests into the engine's running batch without a worker thread each; every
        request is answered on its own when it finishes (``_reply_loop``).  The engine may finish
        a request before ``submit`` returns, so each completion carries its batch's rid table and
        an event set as soon as that table is filled: the reply thread waits for exactly that (no
        timeout that could drop a reply)."""
        from ..engine.sampling import SamplingParams
        table: Dict[int, int] = {}
        ready = threading.Event()
        try:
            try:
                seqs = self.engine.submit(prompts, SamplingParams.from_dict(params or {}),
                                          notify=lambda s_: self._rq.put((s_, table, ready)))
            except Exception as e:  # noqa: BLE001 - report, never kill the submit thread
                for rid in rids:
                    self._safe_reply({"id": rid, "error": f"engine failed: {e}"})
                return
            for s_, rid in zip(seqs, rids):
                table[id(s_)] = rid
        finally:
            ready.set()
        for s_ in seqs:
            if s_.error is not None and s_.done.is_set() and s_.notify is None:   # rejected up front
                self._rq.put((s_, table, ready))

    def _reply_loop(self) -> None:
        while True:
            item = self._rq.get()
            if item is None:
                return
            s_, table, ready = item
            ready.wait()   # set right after engine.submit returns (or raises)
            rid = table.get(id(s_))
            if rid is None:
                continue
            try:
                res = EnginePool.to_payloads(self.engine.results([s_]))[0]
            except Exception as e:  # noqa: BLE001
                res = {"error": f"engine failed: {e}"}
            self._safe_reply({"id": rid, "result": res})

    def serve(self) -> None:
        """Receive until the router sends stop (or disappears)."""
        import os
        self.engine.start()   # background step loop: concurrent requests join one batch
        try:
            while True:
                try:
                    msg = p2p.recv_obj(self.router, self.ctrl, tag=TAG_REQ)
                except Exception:  # router died: stop serving
                    return
                op = msg.get("op")
                if op == "stop":
                    self._dq.put(None)
                    self._sub_ex.shutdown(wait=True)
                    self._ex.shutdown(wait=True)
                    self._rq.put(None)
                    self._rthread.join(timeout=30)
                    self._reply({"op": "bye"})
                    return
                if op == "ping":
                    nd = fault("ping_delay_n", 0, int)
                    if nd > 0:   # fault injection (tests): the first pings stall the receiver loop
                        self._pings_seen = getattr(self, "_pings_seen", 0) + 1
                        if self._pings_seen <= nd:
                            time.sleep(fault("ping_delay_s", 1.0, float))
                    self._reply({"id": msg["id"], "op": "pong",
                                 "stats": {k: v for k, v in self.engine.stats().items()
                                           if isinstance(v, (int, float, str))}})
                elif op == "ping_data":
                    self._dq.put(msg)
                elif op == "sync":
                    self.engine.mirror_control({"sync": True})
                    if self.on_sync is not None:
                        self.on_sync()
                elif op == "generate":
                    if fault("die_on") and any(fault("die_on") in p for p in msg.get("prompts", [])):
                        os._exit(17)   # fault injection (tests): the pool process dies mid-request
                    self._gen_seen = getattr(self, "_gen_seen", 0) + 1
                    die_after, die_rank = fault("die_after", 0, int), fault("die_rank")
                    if die_after and self._gen_seen > die_after and (
                            die_rank is None or int(die_rank) == int(os.environ.get("RANK", "-1"))):
                        os._exit(17)   # fault injection (tests): this leader dies after N requests
                    self._ex.submit(self._generate, msg["id"], msg["prompts"], msg.get("params"))
                elif op == "submit":
                    self._gen_seen = getattr(self, "_gen_seen", 0) + 1
                    die_after, die_rank = fault("die_after", 0, int), fault("die_rank")
                    if die_after and self._gen_seen > die_after and (
                            die_rank is None or int(die_rank) == int(os.environ.get("RANK", "-1"))):
                        os._exit(17)   # fault injection (tests): this leader dies after N requests
                    self._sub_ex.submit(self._submit, msg["ids"], msg["prompts"], msg.get("params"))
                elif op in ("generate_ids", "submit_ids"):
                    self._dq.put(msg)
        finally:
            self._dq.put(None)
            self._rq.put(None)
            self.engine.stop()


class ReplicatedPool(PoolClient):
    """Data-parallel replicas of one tier with least-loaded dispatch."""

    def __init__(self, name: str, replicas: List[PoolClient]):
        super().__init__()
        if not replicas:
            raise ValueError("need at least one replica")
        self.name = name
        self.replicas = replicas
        self.inflight = [0] * len(replicas)
        self._lock = threading.Lock()
        self._ex = ThreadPoolExecutor(max_workers=len(replicas))

    def _state(self, h) -> list:
        """[serving replica, released] of a handle this pool submitted, kept ON the handle (an
        id()-keyed table would leak entries of never-collected handles and could hand a recycled
        id a stale 'released' flag).  Keyed by this pool so nested replicated pools never mix."""
        st = getattr(h, "rp", None)
        if st is None:
            st = {}
            h.rp = st
        return st.setdefault(id(self), [0, False])

    def _pick(self) -> int:
        with self._lock:
            live = [k for k in range(len(self.replicas)) if getattr(self.replicas[k], "alive", True)]
            i = min(live or range(len(self.replicas)), key=lambda k: self.inflight[k])
            self.inflight[i] += 1
            return i

    def process(self, history: Any) -> Dict[str, Any]:
        i = self._pick()
        try:
            return self.replicas[i].process(history)
        finally:
            with self._lock:
                self.inflight[i] -= 1

    def process_batch(self, histories: Sequence[Any]) -> List[Dict[str, Any]]:
        n = len(self.replicas)
        if n == 1 or len(histories) <= 1:
            return self.replicas[0].process_batch(histories) if n == 1 else [self.process(h) for h in histories]
        with self._lock:  # assign round-robin starting from the least-loaded live replica
            live = [k for k in range(n) if getattr(self.replicas[k], "alive", True)] or list(range(n))
            order = sorted(live, key=lambda k: self.inflight[k])
            shards: Dict[int, List[int]] = {k: [] for k in order}
            for j in range(len(histories)):
                shards[order[j % len(order)]].append(j)
            for k, idx in shards.items():
                self.inflight[k] += len(idx)
        futs = {k: self._ex.submit(self.replicas[k].process_batch, [histories[j] for j in idx])
                for k, idx in shards.items() if idx}
        out: List[Any] = [None] * len(histories)
        for k, f in futs.items():
            try:
                res = f.result()
            finally:
                with self._lock:
                    self.inflight[k] -= len(shards[k])
            for j, r in zip(shards[k], res):
                out[j] = r
        return out

    # ------------------------------------------------------------------ non-blocking requests
    def submit_batch(self, histories: Sequence[Any], overrides: Optional[Dict[str, Any]] = None,
                     notify=None, failover: bool = False) -> List[Any]:
        """Shard the requests over the live replicas (least-loaded first, round robin) and submit
        each shard WITHOUT waiting; a replica's load drops as each of its requests completes.
        Replicas without ``submit_batch`` are served on a thread (``ThreadSubmit``)."""
        n = len(self.replicas)
        with self._lock:
            live = [k for k in range(n) if getattr(self.replicas[k], "alive", True)] or list(range(n))
            order = sorted(live, key=lambda k: self.inflight[k])
            shards: Dict[int, List[int]] = {k: [] for k in order}
            for j in range(len(histories)):
                shards[order[j % len(order)]].append(j)
            for k, idx in shards.items():
                self.inflight[k] += len(idx)
        out: List[Any] = [None] * len(histories)
        for k, idx in shards.items():
            if not idx:
                continue
            rep = self.replicas[k]

            def done_cb(h, k=k):
                self._release(h, k)
                if notify is not None:
                    notify(h)
            hs_ = [histories[j] for j in idx]
            sub = getattr(rep, "submit_failover", None) if failover else None
            if sub is not None:
                hs = sub(hs_, notify=done_cb)
            elif getattr(rep, "submit_batch", None) is not None:
                hs = rep.submit_batch(hs_, overrides, notify=done_cb) if overrides else rep.submit_batch(hs_, notify=done_cb)
            else:
                from .base import ThreadSubmit
                hs = ThreadSubmit.submit_batch(rep, hs_, overrides, notify=done_cb)
            for j, h in zip(idx, hs):
                with self._lock:
                    self._state(h)[0] = k
                out[j] = h
            for h in hs:   # finished already, or rejected up front (never notified): counted down now
                if h.done.is_set():
                    self._release(h, k)
        return out

    def _release(self, h, k: int) -> None:
        """A submitted request stopped loading replica k (exactly once per handle)."""
        with self._lock:
            st = self._state(h)
            if st[1]:
                return
            st[1] = True
            self.inflight[k] -= 1

    def submit_failover(self, histories: Sequence[Any], notify=None) -> List[Any]:
        return self.submit_batch(histories, notify=notify, failover=True)

    def collect(self, handles: Sequence[Any]) -> List[Dict[str, Any]]:
        out: List[Any] = [None] * len(handles)
        by: Dict[int, List[int]] = {}
        for j, h in enumerate(handles):
            with self._lock:
                k = self._state(h)[0]
            self._release(h, k)   # idempotent: a later done callback does not count it again
            by.setdefault(k, []).append(j)
        for k, idx in by.items():
            rep = self.replicas[k]
            col = getattr(rep, "collect", None)
            res = col([handles[j] for j in idx]) if col is not None else [handles[j].payload() for j in idx]
            for j, r in zip(idx, res):
                out[j] = r
        return out

    def health(self) -> Dict[str, Any]:
        return {"ok": any(r.health().get("ok") for r in self.replicas), "replicas": len(self.replicas)}
