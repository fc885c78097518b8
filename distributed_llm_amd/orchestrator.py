"""Orchestrator — the ``Router.route_query`` contract (reference L5).

Reference: ``src/router.py:13-319`` (ctor :14-59, ``set_threshold`` :65-67, ``_extract_text``
:73-102, ``_history_to_query_and_context`` :104-147, ``_run_device`` :152-171, response
cache :179-193, ``route_query`` :199-319).

Same contract: ``route_query(history) -> (payload, response_tokens, device)`` with the same
payload keys on a miss and on a response-cache hit.  MI355X-first additions:
  * devices are *pools* (``pools.base.PoolClient``): an in-process GPU engine, an HTTP pool
    worker, or the CPU echo backend; ``.nano`` / ``.orin`` attributes keep the reference
    names for harness compatibility;
  * ``route_batch(histories)`` routes many conversations at once and hands each pool its
    whole group, so the engine batches prefill/decode (continuous batching) instead of
    serving one request at a time;
  * state (response store, perf feedback) is lock-protected;
  * failover can optionally penalise the failed primary in the perf router
    (``"penalise_failed_primary"``, default False = reference behaviour, quirk 3);
  * per-request timing split (queue / prefill / decode / ttft) is surfaced under
    ``payload["timing"]`` when the pool reports it.
"""
from __future__ import annotations

import hashlib
import logging
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

from .config import LARGE, PRODUCTION_CFG, BENCHMARK_CFG, SMALL, other_tier
from .router.query_router import QueryRouter
from .router.tokens import TokenCounter
from .utils.tracing import tracer

logger = logging.getLogger(__name__)


def history_to_query_and_context(history: Sequence[Dict[str, Any]], last_k: int = 6
                                 ) -> Tuple[str, Optional[str], str]:
    """Split history into (latest user query, prior context text, context hash).

    Context lines are ``"role: content"`` for non-empty messages; the hash is
    sha256 over the last ``last_k`` prior messages, first 16 hex chars (reference
    ``router.py:104-147``).
    """
    if not history:
        return "", None, "nohist"
    idx = None
    for i in range(len(history) - 1, -1, -1):
        m = history[i]
        if isinstance(m, dict) and m.get("role") == "user":
            idx = i
            break
    if idx is None:
        query, prior = "", list(history)
    else:
        query, prior = (history[idx].get("content") or "").strip(), list(history[:idx])
    lines = [f"{(m.get('role') or '').strip()}: {(m.get('content') or '').strip()}"
             for m in prior if isinstance(m, dict) and (m.get("content") or "").strip()]
    context = "\n".join(lines) if lines else None
    tail = prior[-last_k:] if last_k > 0 else []
    compact = [f"{m.get('role', '')}:{(m.get('content') or '').strip()}"
               for m in tail if isinstance(m, dict)]
    ctx_hash = hashlib.sha256("\n".join(compact).encode("utf-8")).hexdigest()[:16]
    return query, context, ctx_hash


def extract_text(resp: Any) -> Optional[str]:
    """Normalise any pool response shape into text (reference ``router.py:73-102``)."""
    if resp is None:
        return None
    if isinstance(resp, str):
        return resp.strip() or None
    if isinstance(resp, dict):
        for key in ("response", "content", "message"):
            v = resp.get(key)
            if isinstance(v, str) and v.strip():
                return v.strip()
            if isinstance(v, dict):
                inner = v.get("content")
                if isinstance(inner, str) and inner.strip():
                    return inner.strip()
        if "error" in resp:
            parts = [str(resp.get(k, "")).strip() for k in ("error", "detail", "body")]
            joined = " ".join(p for p in parts if p)
            return joined[:300] if joined else None
    return None


def is_error(raw: Any) -> bool:
    return isinstance(raw, dict) and "error" in raw


class Router:
    def __init__(self, strategy: str = "hybrid", config: Optional[Dict[str, Any]] = None,
                 threshold_fallback: int = 100, benchmark_mode: bool = False,
                 pools: Optional[Dict[str, Any]] = None):
        self.token_counter = TokenCounter()
        self.threshold_fallback = threshold_fallback
        self.benchmark_mode = benchmark_mode
        if config is not None:
            self.config = config
        else:
            self.config = BENCHMARK_CFG if benchmark_mode else PRODUCTION_CFG
        self.query_router = QueryRouter(strategy=strategy, config=self.config)
        self.enable_response_cache = (not benchmark_mode
                                      and bool(self.config.get("enable_response_cache", False)))
        self.cache_last_k = int(self.config.get("cache_last_k", 6))
        self.enable_failover = bool(self.config.get("enable_failover", True))
        self.penalise_failed_primary = bool(self.config.get("penalise_failed_primary", False))
        self.tokens_from_engine = bool(self.config.get("tokens_from_engine", False))
        self.pool_health: Dict[str, Dict[str, Any]] = {}
        self._responses: Dict[str, Dict[str, Any]] = {}
        self._lock = threading.RLock()
        if pools is None:
            from .pools.base import default_pools
            pools = default_pools(self.config)
        self.pools = {SMALL: pools[SMALL], LARGE: pools[LARGE]}

    # reference attribute names
    @property
    def nano(self):
        return self.pools[SMALL]

    @property
    def orin(self):
        return self.pools[LARGE]

    def set_threshold(self, threshold: int) -> None:
        self.threshold_fallback = threshold

    # ------------------------------------------------------------------ helpers
    def _split(self, history):
        return history_to_query_and_context(history, self.cache_last_k)

    def _response_key(self, query: str) -> str:
        # Context-independent key, as in the reference (quirk 2); "response_cache_context": True
        # opts into context-aware keys.
        return f"{self.query_router.strategy}|{query.lower().strip()}"

    def _decide(self, query: str, context: Optional[str], ctx_hash: str, history) -> Dict[str, Any]:
        t0 = time.perf_counter()
        try:
            with tracer.span("route.decide", "router") as targs:
                d = self.query_router.route_query(query=query, context=context, context_key=ctx_hash)
                targs.update(device=d.device, method=d.method, cache_hit=bool(d.cache_hit))
            out = {"device": d.device, "method": d.method, "confidence": float(d.confidence),
                   "reasoning": d.reasoning, "cache_hit": d.cache_hit}
        except Exception as exc:
            size = self.token_counter.get_context_size(history)
            dev = LARGE if size > self.threshold_fallback else SMALL
            out = {"device": dev, "method": "fallback_ctx_size", "confidence": 0.2,
                   "reasoning": (f"router failed: {exc}; ctx_size={size}, "
                                 f"threshold_fallback={self.threshold_fallback}"),
                   "cache_hit": False}
        out["overhead_ms"] = (time.perf_counter() - t0) * 1000.0
        return out

    def _cached_payload(self, query: str):
        if not self.enable_response_cache:
            return None
        with self._lock:
            c = self._responses.get(self._response_key(query))
        if c is None:
            return None
        text, which = c.get("text", ""), c.get("device", SMALL)
        toks = self.token_counter.count_tokens({"role": "assistant", "content": text})
        return ({"response": text, "raw": c.get("raw"), "cache_hit": True,
                 "routing_method": "response_cache", "routing_confidence": 1.0,
                 "routing_reasoning": f"response cache hit -> {which}",
                 "routing_overhead_ms": 0.0, "ok": True}, toks, which)

    def _finish(self, query: str, dec: Dict[str, Any], raw: Any, which: str, lat_ms: float,
                primary_failed: Optional[str] = None):
        text = extract_text(raw) or "No response available"
        ntok = raw.get("num_tokens") if isinstance(raw, dict) else None
        # reference: response tokens = TokenCounter over the returned text (src/router.py:286);
        # ``tokens_from_engine`` reports the engine's generated-token count instead (bench.py:
        # throughput in generated tokens), and the payload carries both
        counted = self.token_counter.count_tokens({"role": "assistant", "content": text})
        toks = int(ntok) if (ntok is not None and self.tokens_from_engine) else counted
        ok = not is_error(raw)
        try:
            self.query_router.update_perf(which, lat_ms, toks, ok=ok)
            if primary_failed and self.penalise_failed_primary:
                self.query_router.update_perf(primary_failed, lat_ms, 0, ok=False)
        except Exception:
            pass
        if self.enable_response_cache:
            with self._lock:
                self._responses[self._response_key(query)] = {
                    "text": text, "raw": raw, "device": which,
                    "routing_confidence": round(dec["confidence"], 4)}
        payload = {"response": text, "raw": raw, "cache_hit": False,
                   "benchmark_mode": self.benchmark_mode,
                   "routing_overhead_ms": round(dec["overhead_ms"], 2),
                   "routing_method": dec["method"],
                   "routing_confidence": round(dec["confidence"], 4),
                   "routing_reasoning": dec["reasoning"], "ok": ok}
        if primary_failed:
            payload["failover_from"] = primary_failed   # the decided tier failed; ``which`` served it
        if isinstance(raw, dict) and "timing" in raw:
            payload["timing"] = dict(raw["timing"], generated_tokens=ntok, counted_tokens=counted)
        return payload, toks, which

    def on_pool_health(self, name: str, ok: bool, rtt_us: Optional[float]) -> None:
        """Sink for periodic pool health probes (pools.remote.RemotePool.start_probes): the last
        state per pool is kept for /metrics and a FAILED probe is fed to the perf router as a
        failed request (its failure-rate penalty, query_router_engine.py:442-445), so a pool that
        stops answering loses traffic before a user request has to time out on it."""
        with self._lock:
            st = self.pool_health.setdefault(name, {"ok": True, "probes": 0, "failures": 0, "rtt_us": None})
            st["probes"] += 1
            st["ok"] = bool(ok)
            if ok:
                st["rtt_us"] = rtt_us
            else:
                st["failures"] += 1
        if not ok:
            try:
                self.query_router.update_perf(name, 5000.0, 0, ok=False)
            except Exception:  # noqa: BLE001
                pass

    def _pool_down(self, device: str) -> bool:
        """A pool known to be out of service (a remote pool whose process died or that failed its
        health probes: ``alive`` False) while the other tier's pool is up: requests decided for it
        go straight to the other tier as a failover instead of paying a failed attempt first."""
        if not self.enable_failover:
            return False
        pool, other = self.pools.get(device), self.pools.get(other_tier(device))
        return (pool is not None and getattr(pool, "alive", True) is False
                and other is not None and getattr(other, "alive", True) is not False)

    def _run(self, device: str, history, failover: bool = False) -> Tuple[Any, str, float]:
        t0 = time.perf_counter()
        try:
            with tracer.span("pool.process", "pool", device=device, failover=failover):
                pool = self.pools[device]
                # a failover to a remote pool hands the prompt over as token ids (pools.remote)
                fn = getattr(pool, "process_failover", None) if failover else None
                raw = fn(history) if fn is not None else pool.process(history)
        except Exception as exc:  # a pool that raises is an error response, not a crash
            raw = {"error": f"pool {device} failed: {exc}"}
        return raw, device, (time.perf_counter() - t0) * 1000.0

    # ------------------------------------------------------------------ public API
    def route_query(self, conversation_history: List[Dict[str, Any]]):
        query, context, ctx_hash = self._split(conversation_history)
        hit = self._cached_payload(query)
        if hit is not None:
            return hit
        dec = self._decide(query, context, ctx_hash, conversation_history)
        if self._pool_down(dec["device"]):
            raw, which, lat = self._run(other_tier(dec["device"]), conversation_history, failover=True)
            return self._finish(query, dec, raw, which, lat, dec["device"])
        raw, which, lat = self._run(dec["device"], conversation_history)
        failed = None
        if self.enable_failover and is_error(raw):
            raw2, which2, lat2 = self._run(other_tier(which), conversation_history, failover=True)
            if not is_error(raw2):
                failed = which
                raw, which, lat = raw2, which2, lat2
        return self._finish(query, dec, raw, which, lat, failed)

    def route_batch(self, histories: Sequence[List[Dict[str, Any]]]):
        """Route a batch of independent conversations; each pool serves its group batched.

        Returns a list of ``(payload, response_tokens, device)`` in input order.  Latency per
        request is the pool's per-request latency (queue + prefill + decode), as reported.
        """
        results: List[Any] = [None] * len(histories)
        groups: Dict[str, List[int]] = {SMALL: [], LARGE: []}
        meta: Dict[int, Tuple[str, Dict[str, Any]]] = {}
        splits = [self._split(h) for h in histories]
        self._prefetch_embeddings([sp[0] for sp in splits], [sp[2] for sp in splits])
        for i, (h, (query, context, ctx_hash)) in enumerate(zip(histories, splits)):
            hit = self._cached_payload(query)
            if hit is not None:
                results[i] = hit
                continue
            dec = self._decide(query, context, ctx_hash, h)
            meta[i] = (query, dec)
            groups[dec["device"]].append(i)
        failed: Dict[int, str] = {}
        for dev in (SMALL, LARGE):   # a tier that is down: its turns go to the other tier up front
            if groups[dev] and self._pool_down(dev):
                for i in groups[dev]:
                    failed[i] = dev
                groups[other_tier(dev)].extend(groups[dev])
                groups[dev] = []
        retry: Dict[str, List[int]] = {SMALL: [], LARGE: []}
        raws: Dict[int, Tuple[Any, str, float]] = {}
        for dev, outs in self._process_groups(groups, histories).items():
            for i, (raw, lat) in zip(groups[dev], outs):
                raws[i] = (raw, dev, lat)
                if self.enable_failover and is_error(raw) and i not in failed:
                    retry[other_tier(dev)].append(i)
        if any(retry.values()):
            for dev, outs in self._process_groups(retry, histories).items():
                for i, (raw, lat) in zip(retry[dev], outs):
                    if not is_error(raw):
                        failed[i] = raws[i][1]
                        raws[i] = (raw, dev, lat)
        for i, (query, dec) in meta.items():
            raw, which, lat = raws[i]
            results[i] = self._finish(query, dec, raw, which, lat, failed.get(i))
        return results

    # ------------------------------------------------------------------ turn pipelining
    def _decide_batch(self, histories: Sequence[List[Dict[str, Any]]]) -> List[Tuple[str, Any, Any]]:
        """Routing half of ``route_batch``: ("hit", payload, None) for a response-cache hit,
        else ("route", query, decision)."""
        splits = [self._split(h) for h in histories]
        self._prefetch_embeddings([sp[0] for sp in splits], [sp[2] for sp in splits])
        out: List[Tuple[str, Any, Any]] = []
        for h, (query, context, ctx_hash) in zip(histories, splits):
            hit = self._cached_payload(query)
            if hit is not None:
                out.append(("hit", hit, None))
            else:
                out.append(("route", query, self._decide(query, context, ctx_hash, h)))
        return out

    def route_concurrent(self, conversation_history: List[Dict[str, Any]]):
        """``route_query`` for many concurrent callers (one thread per conversation).

        Routing decisions of callers that arrive while a decision batch is in flight are made
        together (one batched encoder forward, ``pools.base.Coalescer``); each request is then
        served on its own, so with an engine running its background loop (``LLMEngine.start``)
        it joins the running continuous batch and its caller resumes as soon as ITS answer is
        done — no conversation waits for another conversation's generation (unlike
        ``route_batch``, whose callers all wait for the slowest member of the batch)."""
        with self._lock:
            dc = getattr(self, "_decider", None)
            if dc is None:
                from .pools.base import Coalescer
                dc = self._decider = Coalescer(self._decide_batch)
        kind, a, dec = dc.submit([conversation_history])[0]
        if kind == "hit":
            return a
        query = a
        raw, which, lat = self._run(dec["device"], conversation_history)
        failed = None
        if self.enable_failover and is_error(raw):
            raw2, which2, lat2 = self._run(other_tier(which), conversation_history, failover=True)
            if not is_error(raw2):
                failed = which
                raw, which, lat = raw2, which2, lat2
        if isinstance(raw, dict) and "latency_ms" in raw:
            lat = float(raw["latency_ms"])
        return self._finish(query, dec, raw, which, lat, failed)

    # ------------------------------------------------------------------ event-driven dispatch
    def dispatch_batch(self, histories: Sequence[List[Dict[str, Any]]],
                       notify: Optional[Callable[[Any], None]] = None) -> List[Dict[str, Any]]:
        """Route a batch of conversations (one batched decision pass) and SUBMIT each request to
        its tier without waiting: pools with a non-blocking ``submit_batch`` (in-process engines
        running their background loop) return handles; other pools are served synchronously here.
        Returns one ticket per history; ``ticket_done`` / ``finish_ticket`` complete them.  A
        single client thread can keep hundreds of independent conversations in flight this way
        (each conversation still strictly sequential), instead of one blocked thread each.
        ``notify(handle)`` is called when a submitted ticket's handle (``ticket["handle"]``)
        finishes, so the client can block on a completion queue instead of polling every ticket.
        Tickets without a handle, and requests a pool rejected up front, come back done and are
        never notified; a handle can finish (and be notified) before this returns."""
        tickets: List[Dict[str, Any]] = []
        groups: Dict[str, List[int]] = {SMALL: [], LARGE: []}
        t0 = time.perf_counter()
        for i, (kind, a, dec) in enumerate(self._decide_batch(histories)):
            t: Dict[str, Any] = {"history": histories[i], "t0": t0}
            if kind == "hit":
                t["payload"] = a
                t["latency_ms"] = (time.perf_counter() - t0) * 1000.0
            else:
                t["query"], t["dec"], t["device"] = a, dec, dec["device"]
                if self._pool_down(dec["device"]):   # a tier known to be down: fail over up front
                    t["failover_from"], t["device"] = dec["device"], other_tier(dec["device"])
                    # a double failure then reports the primary's error with no failover, as route_query
                    t["primary_error"] = {"error": f"pool {dec['device']} unavailable"}
                groups[t["device"]].append(i)
            tickets.append(t)
        for dev, idx in groups.items():
            if not idx:
                continue
            self._submit_tickets(dev, [tickets[i] for i in idx], notify)
        return tickets

    def _submit_tickets(self, dev: str, tickets: List[Dict[str, Any]], notify) -> None:
        """Hand tickets to pool ``dev`` without waiting where it can (``submit_batch``; a failover
        ticket goes by ``submit_failover`` - token ids over the data plane to a remote pool - when
        the pool has it); a pool with only the blocking API is served here."""
        pool = self.pools[dev]
        hs = [t["history"] for t in tickets]
        fo = all("failover_from" in t for t in tickets)
        sub = (getattr(pool, "submit_failover", None) if fo else None) or getattr(pool, "submit_batch", None)
        if sub is not None:
            try:
                handles = sub(hs) if notify is None else sub(hs, notify=notify)
            except Exception as exc:  # noqa: BLE001 - a pool that raises: error payloads, done now
                for t in tickets:
                    t.pop("handle", None)
                    t["raw"] = {"error": f"pool {dev} failed: {exc}"}
                return
            for t, h in zip(tickets, handles):
                t["handle"] = h
                t.pop("raw", None)
        else:
            for t in tickets:
                raw, _, _ = self._run(dev, t["history"], failover="failover_from" in t)
                t.pop("handle", None)
                t["raw"] = raw

    @staticmethod
    def ticket_done(t: Dict[str, Any]) -> bool:
        h = t.get("handle")
        return h is None or h.done.is_set()

    def finish_ticket(self, t: Dict[str, Any], notify: Optional[Callable[[Any], None]] = None):
        """(payload, response_tokens, device) of a done ticket: perf feedback, failover to the
        other tier on an error, response-cache store — as ``route_query``.

        Failover is non-blocking when the client passes its completion sink (``notify``) and the
        other tier's pool can submit: the request is re-submitted there and this returns ``None``
        (the ticket is in flight again, under its new ``handle``; finish it once more when that is
        done), so one failed turn never stalls the client's other conversations (the reference
        fails over on the request's own thread, src/router.py:277-282).  Otherwise (no sink, a
        blocking pool) the failover generation runs here, as before.  ``t["latency_ms"]`` is set to
        the client-side turn latency: dispatch to completion, failover included (the reference
        harness times the whole ``route_query``, routing_chatbot_tester.py:408-442)."""
        if "payload" in t:
            return t["payload"]
        which = t["device"]
        if "handle" in t:
            raw = self.pools[which].collect([t["handle"]])[0]
        else:
            raw = t["raw"]
        lat = float(raw["latency_ms"]) if isinstance(raw, dict) and "latency_ms" in raw else \
            (time.perf_counter() - t["t0"]) * 1000.0
        failed = t.get("failover_from")
        if self.enable_failover and is_error(raw) and failed is None:
            other = other_tier(which)
            pool = self.pools[other]
            if notify is not None and (getattr(pool, "submit_failover", None) or getattr(pool, "submit_batch", None)):
                t["failover_from"], t["device"] = which, other
                t["primary_error"] = raw
                self._submit_tickets(other, [t], notify)
                if "handle" in t:
                    return None   # in flight on the other tier
                return self.finish_ticket(t, notify)   # the pool refused it at once: finish now
            raw2, which2, lat2 = self._run(other, t["history"], failover=True)
            if not is_error(raw2):
                failed = which
                raw, which, lat = raw2, which2, lat2
        elif failed is not None and is_error(raw) and "primary_error" in t:
            # the failover failed too: report the primary's error, no failover (as route_query)
            raw, which, failed = t["primary_error"], failed, None
        t["latency_ms"] = (time.perf_counter() - t["t0"]) * 1000.0
        return self._finish(t["query"], t["dec"], raw, which, lat, failed)

    def _prefetch_embeddings(self, queries: List[str], context_keys: Optional[List[str]] = None) -> None:
        """One batched encoder forward for every query of a batch (the GPU encoder keeps it for the
        batch's own lookups even with its memo off), so the semantic router and the semantic cache
        do no per-query encoder launches; then the batch's centroid scores and its semantic-cache
        lookups are scored in one launch each (``prefetch_scores``, ``prefetch_cache``)."""
        emb = self.query_router.cache_embedder
        needs = self.query_router.cache_enabled or self.query_router.strategy in ("semantic", "hybrid")
        if emb is None or not needs or not queries:
            return
        enc = getattr(emb, "prefetch", None) or getattr(emb, "encode_tensor", None) or emb.encode
        try:
            enc(list(dict.fromkeys(queries)))
            self.query_router.prefetch_scores(queries)
            if context_keys is not None:
                self.query_router.prefetch_cache(queries, context_keys)
        except Exception as exc:  # routing still works, just unbatched
            logger.warning("batched embedding prefetch failed: %s", exc)

    def _process_groups(self, groups: Dict[str, List[int]], histories) -> Dict[str, List[Tuple[Any, float]]]:
        """Serve every tier's group (tiers sharing one engine run as ONE continuous batch)."""
        from .pools.factory import dispatch_groups
        hs = {dev: [histories[i] for i in idxs] for dev, idxs in groups.items() if idxs}
        t0 = time.perf_counter()
        try:
            with tracer.span("pool.dispatch_groups", "pool", **{dev: len(h) for dev, h in hs.items()}):
                res = dispatch_groups(self.pools, hs)
        except Exception as exc:
            res = {dev: [{"error": f"pool {dev} failed: {exc}"}] * len(h) for dev, h in hs.items()}
        wall = (time.perf_counter() - t0) * 1000.0
        out: Dict[str, List[Tuple[Any, float]]] = {}
        for dev, raws in res.items():
            out[dev] = [(r, float(r.get("latency_ms", wall)) if isinstance(r, dict) else wall) for r in raws]
        return out
