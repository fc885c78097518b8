"""Predictive routing cache: exact + semantic lookup, recency-weighted device prediction.

Behavioural spec: reference ``src/cache.py`` —
  RoutingRecord :53-77, CacheEntry :79-176 (predict_device :106-140), CacheLookupResult
  :179-192, QueryCache :199-554 (lookup :236-326, insert :328-370, invalidate :372-396,
  warm_up :398-420, save/load :426-465, stats :471-500, clear :502-512, eviction :532-554).

MI355X-first differences:
  * The reference scans every entry in a Python loop per lookup (O(N) cosine in the
    interpreter).  Here embeddings live in a slot-indexed ``EmbeddingIndex`` — a contiguous
    [capacity, dim] table with per-slot norms and context-key ids.  On a GPU box the table is
    an HBM tensor and lookup is ONE fused HIP kernel (mask by context id, cosine, arg-max over
    ≥ threshold) — ``ops.masked_cosine_argmax``; on CPU it is a vectorised numpy GEMV.  A
    288 GB device holds ~180M fp32 384-d entries, so ``cache_max_size`` is no longer a memory
    concern.
  * All counters are updated under the lock (the reference increments ``_attempts`` outside it,
    SURVEY §2.11 quirk 8).
JSON persistence format is identical to the reference's ``CacheEntry.to_dict``.
"""
from __future__ import annotations

import hashlib
import heapq
import itertools
import json
import logging
import re
import threading
from collections import OrderedDict
from dataclasses import dataclass, field
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from ..config import LARGE, SMALL

logger = logging.getLogger(__name__)

PREDICTION_CONFIDENCE_THRESHOLD = 0.60
RECENCY_DECAY = 0.85
MAX_HISTORY = 20


@dataclass
class RoutingRecord:
    device: str
    confidence: float
    method: str
    timestamp: str

    def to_dict(self) -> Dict[str, Any]:
        return {"device": self.device, "confidence": self.confidence,
                "method": self.method, "timestamp": self.timestamp}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "RoutingRecord":
        return cls(device=d["device"], confidence=float(d["confidence"]),
                   method=d.get("method", "unknown"),
                   timestamp=d.get("timestamp", datetime.now().isoformat()))


@dataclass
class CacheEntry:
    query: str
    query_hash: str
    context_key: str
    embedding: Optional[np.ndarray]
    timestamp: datetime
    device_used: str
    response_time: Optional[float] = None
    hit_count: int = 0
    routing_history: List[RoutingRecord] = field(default_factory=list)
    slot: int = -1  # row in the EmbeddingIndex (-1: no embedding)

    MAX_HISTORY = MAX_HISTORY

    def record_routing(self, device: str, confidence: float, method: str) -> None:
        self.routing_history.append(
            RoutingRecord(device, confidence, method, datetime.now().isoformat()))
        if len(self.routing_history) > MAX_HISTORY:
            del self.routing_history[:-MAX_HISTORY]
        self.device_used = device

    def predict_device(self) -> Tuple[str, float]:
        """Recency-decayed (0.85^i, newest first) confidence-weighted vote; large wins ties."""
        if not self.routing_history:
            return self.device_used, 0.5
        small = large = 0.0
        w = 1.0
        for rec in reversed(self.routing_history):
            v = w * rec.confidence
            if rec.device == LARGE:
                large += v
            else:
                small += v
            w *= RECENCY_DECAY
        total = small + large
        if total < 1e-9:
            return self.device_used, 0.5
        if large >= small:
            return LARGE, float(min(large / total, 1.0))
        return SMALL, float(min(small / total, 1.0))

    def to_dict(self) -> Dict[str, Any]:
        return {
            "query": self.query,
            "query_hash": self.query_hash,
            "context_key": self.context_key,
            "embedding": _host_vec(self.embedding).tolist() if self.embedding is not None else None,
            "timestamp": self.timestamp.isoformat(),
            "device_used": self.device_used,
            "response_time": self.response_time,
            "hit_count": self.hit_count,
            "routing_history": [r.to_dict() for r in self.routing_history],
        }

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "CacheEntry":
        emb = d.get("embedding")
        return cls(
            query=d["query"], query_hash=d["query_hash"], context_key=d["context_key"],
            embedding=np.asarray(emb, dtype=np.float32) if emb else None,
            timestamp=datetime.fromisoformat(d["timestamp"]), device_used=d["device_used"],
            response_time=d.get("response_time"), hit_count=d.get("hit_count", 0),
            routing_history=[RoutingRecord.from_dict(r) for r in d.get("routing_history", [])])


@dataclass
class CacheLookupResult:
    entry: CacheEntry
    predicted_device: str
    predicted_confidence: float
    use_hybrid_fallback: bool


def _host_vec(x) -> np.ndarray:
    """An entry's embedding (host array or device tensor) as a flat f32 numpy vector."""
    if hasattr(x, "detach"):
        return x.detach().float().cpu().numpy().reshape(-1)
    return np.asarray(x, dtype=np.float32).reshape(-1)


class EmbeddingIndex:
    """Slot-indexed embedding table for vectorised / on-GPU semantic lookup.

    ``device=None`` keeps a numpy table on the host (vectorised numpy scoring).  A torch device
    string keeps an HBM table [capacity, dim] f32 plus one context id per row, and:
      * row writes are DEFERRED: ``put`` / ``remove`` only record (slot -> vector, context id);
        ``flush`` applies every pending write in one ``ops.cache_write`` launch per 64 rows right
        before the next scoring launch (no copy launch, norm reduction or host sync per insert);
      * a lookup scores only rows of its context (``ops.cache_scan``: context ids read as 16-B
        vectors, matching rows fetched and scored), and ``best_batch`` scores a whole routing
        batch in one launch with one read-back.
    ``dirty`` collects the context ids whose rows changed since the owner last cleared it (the
    routing cache's batch prefetch uses it to know which prefetched results are still exact).
    """

    def __init__(self, dim: int = 384, capacity: int = 1024, device: Optional[str] = None):
        self.dim = dim
        self.device = device
        self._free: List[int] = []
        self._next = 0
        # context key -> small int id stored per slot; ids are reference-counted by the slots that
        # hold them and recycled when the last slot goes (TTL / LRU eviction, replacement), so a
        # long-running server does not keep one entry per routed turn forever
        self._ctx_ids: Dict[str, int] = {}
        self._ctx_key: Dict[int, str] = {}
        self._ctx_refs: Dict[int, int] = {}
        self._free_cids: List[int] = []
        self._slot_cid: Dict[int, int] = {}
        self._pending: Dict[int, Tuple[Any, int]] = {}   # device mode: slot -> (vector | None, ctx id)
        self.dirty: set = set()
        self.track_dirty = False                          # on while a batch prefetch is outstanding
        self.launches = {"write": 0, "scan": 0}           # device launches issued (bench / tests)
        self._alloc(capacity)

    def _alloc(self, capacity: int) -> None:
        self.capacity = capacity
        if self.device is None:
            self.table = np.zeros((capacity, self.dim), dtype=np.float32)
            self.norms = np.zeros(capacity, dtype=np.float32)
            self.ctx = np.full(capacity, -1, dtype=np.int32)
        else:
            import torch
            self.table = torch.zeros((capacity, self.dim), dtype=torch.float32, device=self.device)
            self.norms = None     # the GPU scorer computes row norms from the row it loads
            self.ctx = torch.full((capacity,), -1, dtype=torch.int32, device=self.device)

    def _grow(self) -> None:
        self.flush()
        old_t, old_n, old_c, old_cap = self.table, self.norms, self.ctx, self.capacity
        self._alloc(old_cap * 2)
        self.table[:old_cap] = old_t
        if old_n is not None:
            self.norms[:old_cap] = old_n
        self.ctx[:old_cap] = old_c

    def ctx_id(self, key: str) -> int:
        i = self._ctx_ids.get(key)
        if i is None:
            i = self._free_cids.pop() if self._free_cids else len(self._ctx_ids)
            self._ctx_ids[key] = i
            self._ctx_key[i] = key
            self._ctx_refs[i] = 0
        return i

    def cid_of(self, key: str) -> Optional[int]:
        return self._ctx_ids.get(key)

    def _release(self, slot: int) -> None:
        cid = self._slot_cid.pop(slot, None)
        if cid is None:
            return
        if self.track_dirty:
            self.dirty.add(cid)
        self._ctx_refs[cid] -= 1
        if self._ctx_refs[cid] == 0:
            del self._ctx_refs[cid]
            del self._ctx_ids[self._ctx_key.pop(cid)]
            self._free_cids.append(cid)

    def num_contexts(self) -> int:
        return len(self._ctx_ids)

    def put(self, vec: Any, context_key: str, slot: int = -1) -> int:
        if slot < 0:
            if self._free:
                slot = self._free.pop()
            else:
                if self._next >= self.capacity:
                    self._grow()
                slot = self._next
                self._next += 1
        self._release(slot)          # a replaced slot drops its old context reference
        cid = self.ctx_id(context_key)
        self._ctx_refs[cid] += 1
        self._slot_cid[slot] = cid
        if self.track_dirty:
            self.dirty.add(cid)
        if self.device is None:
            v = np.asarray(vec, dtype=np.float32).reshape(-1)
            self.table[slot] = v
            self.norms[slot] = float(np.linalg.norm(v))
            self.ctx[slot] = cid
        else:
            import torch
            if isinstance(vec, torch.Tensor):   # device vector: referenced until the next flush
                v = vec.reshape(-1)
                if v.device != self.table.device or v.dtype != torch.float32 or not v.is_contiguous():
                    v = v.to(self.table.device, torch.float32).contiguous()
            else:
                v = torch.from_numpy(np.asarray(vec, dtype=np.float32).reshape(-1).copy()).to(self.table.device)
            self._pending[slot] = (v, cid)
        return slot

    def remove(self, slot: int) -> None:
        if slot < 0:
            return
        if self.device is None:
            self.ctx[slot] = -1
        else:
            self._pending[slot] = (None, -1)
        self._release(slot)
        self._free.append(slot)

    def flush(self) -> None:
        """Apply the deferred device writes (one launch per 64 rows)."""
        if not self._pending:
            return
        from .. import ops
        writes = [(slot, v, cid) for slot, (v, cid) in self._pending.items()]
        self._pending.clear()
        ops.cache_write(writes, self.table, self.ctx)
        self.launches["write"] += -(-len(writes) // ops.CACHE_WRITE_MAX)

    def clear(self) -> None:
        self._free.clear()
        self._next = 0
        self._ctx_ids.clear()
        self._ctx_key.clear()
        self._ctx_refs.clear()
        self._free_cids.clear()
        self._slot_cid.clear()
        self._pending.clear()
        self.dirty.clear()
        if self.device is None:
            self.ctx[:] = -1
        else:
            self.ctx.fill_(-1)

    def _best_host(self, q: Any, cid: int, threshold: float) -> Tuple[int, float]:
        hi = self._next
        qv = np.asarray(q, dtype=np.float32).reshape(-1)
        nq = float(np.linalg.norm(qv))
        if nq < 1e-9:
            return -1, 0.0
        mask = (self.ctx[:hi] == cid) & (self.norms[:hi] >= 1e-9)
        if not mask.any():
            return -1, 0.0
        idx = np.nonzero(mask)[0]
        sims = (self.table[idx] @ qv) / (self.norms[idx] * nq)
        j = int(np.argmax(sims))
        s = float(sims[j])
        return (int(idx[j]), s) if s >= threshold else (-1, 0.0)

    def best(self, q: Any, context_key: str, threshold: float) -> Tuple[int, float]:
        """Best slot with cosine >= threshold among slots of ``context_key``; (-1, 0) if none."""
        return self.best_batch([q], [context_key], threshold)[0]

    def best_batch(self, qs: List[Any], context_keys: List[str], threshold: float) -> List[Tuple[int, float]]:
        """``best`` for a whole routing batch: on the GPU one scoring launch (per 128 queries) and
        ONE read-back; queries whose context has no rows are answered on the host."""
        out: List[Tuple[int, float]] = [(-1, 0.0)] * len(qs)
        todo = [(i, self._ctx_ids.get(ck)) for i, ck in enumerate(context_keys)]
        todo = [(i, cid) for i, cid in todo if cid is not None and qs[i] is not None]
        if not todo or self._next == 0:
            return out
        if self.device is None:
            for i, cid in todo:
                out[i] = self._best_host(qs[i], cid, threshold)
            return out
        from .. import ops
        import torch
        self.flush()
        qv = []
        for i, _ in todo:
            q = qs[i]
            if not isinstance(q, torch.Tensor):
                q = torch.from_numpy(np.asarray(q, dtype=np.float32).reshape(-1).copy())
            qv.append(q.reshape(-1).to(self.table.device, torch.float32))
        res = ops.cache_scan(qv, [cid for _, cid in todo], self.table, self.ctx, self._next, threshold)
        self.launches["scan"] += -(-len(qv) // ops.CACHE_SCAN_MAX_Q)
        for (i, _), r in zip(todo, res):
            out[i] = r
        return out


class QueryCache:
    """Thread-safe LRU + TTL routing cache with semantic lookup and device prediction."""

    def __init__(self, max_size: int = 100, ttl_seconds: int = 300, similarity_threshold: float = 0.85,
                 use_semantic: bool = True,
                 prediction_confidence_threshold: float = PREDICTION_CONFIDENCE_THRESHOLD,
                 index_device: Optional[str] = None, dim: int = 384):
        self.max_size = max_size
        self.ttl_seconds = ttl_seconds
        self.similarity_threshold = similarity_threshold
        self.use_semantic = use_semantic
        self.prediction_confidence_threshold = prediction_confidence_threshold
        self._store: "OrderedDict[str, CacheEntry]" = OrderedDict()
        self._lock = threading.RLock()
        self._index = EmbeddingIndex(dim=dim, capacity=max(64, min(max_size, 1 << 20)),
                                     device=index_device)
        self._slot_to_hash: Dict[int, str] = {}
        # expiry heap (timestamp, seq, hash) with lazy deletion: TTL eviction pops only expired
        # records instead of scanning every entry on every lookup (the reference's O(N) sweep,
        # cache.py:250,532-538, was ~0.25 s per 256-conversation step at 1e4 entries)
        self._expiry: List[Tuple[datetime, int, str]] = []
        self._seq = itertools.count()
        self._hits = 0
        self._attempts = 0
        self._evictions = 0
        self._hybrid_fallbacks = 0
        # batch prefetch (``prefetch``): (query, context_key) -> (slot, sim) scored together
        self._pre: Dict[Tuple[str, str], Tuple[int, float]] = {}
        self.prefetch_used = 0       # semantic lookups answered from a batch prefetch
        self.prefetch_fallbacks = 0  # ... re-scored on their own (their context changed meanwhile)

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _make_hash(query: str, context_key: str) -> str:
        return hashlib.md5(f"{context_key}||{query.lower().strip()}".encode("utf-8")).hexdigest()

    def _is_valid(self, entry: CacheEntry, now: Optional[datetime] = None) -> bool:
        return ((now or datetime.now()) - entry.timestamp).total_seconds() <= self.ttl_seconds

    def _delete_entry(self, h: str) -> None:
        e = self._store.pop(h, None)
        if e is not None and e.slot >= 0:
            self._index.remove(e.slot)
            self._slot_to_hash.pop(e.slot, None)
            e.slot = -1

    def _set_embedding(self, e: CacheEntry, emb: Optional[np.ndarray]) -> None:
        if emb is None:
            return
        if hasattr(emb, "detach") and self._index.device is not None:
            # device embedding into the HBM index: stays on the GPU (no host round trip per insert).
            # The encoder's rows are never written again (each forward allocates its output), so the
            # entry keeps a reference, not a copy; converted to host only by save / to_dict
            arr = emb.detach().reshape(-1)
            if arr.device != self._index.table.device or arr.dtype != self._index.table.dtype:
                arr = arr.to(self._index.table.device, dtype=self._index.table.dtype)
        else:
            arr = np.asarray(emb.detach().float().cpu().numpy() if hasattr(emb, "detach") else emb,
                             dtype=np.float32).reshape(-1).copy()
        e.embedding = arr
        if e.slot < 0 or self._slot_to_hash.get(e.slot) != e.query_hash:
            e.slot = self._index.put(arr, e.context_key)
            self._slot_to_hash[e.slot] = e.query_hash
        else:
            self._index.put(arr, e.context_key, slot=e.slot)

    def _stamp(self, e: CacheEntry, ts: Optional[datetime] = None) -> None:
        e.timestamp = ts or datetime.now()
        heapq.heappush(self._expiry, (e.timestamp, next(self._seq), e.query_hash))

    def _pop_expired(self, now: datetime, limit: Optional[int] = None) -> int:
        """Delete expired entries in expiry order (stale heap records are skipped)."""
        n = 0
        while self._expiry and (limit is None or n < limit):
            ts, _, h = self._expiry[0]
            if (now - ts).total_seconds() <= self.ttl_seconds:
                break
            heapq.heappop(self._expiry)
            e = self._store.get(h)
            if e is not None and e.timestamp == ts:
                self._delete_entry(h)
                self._evictions += 1
                n += 1
        return n

    def _evict_expired(self) -> None:
        with self._lock:
            self._pop_expired(datetime.now())

    def _evict_one(self) -> None:
        # stale first (reference cache.py:540-554), then least recently used
        if self._pop_expired(datetime.now(), limit=1):
            return
        if self._store:
            self._delete_entry(next(iter(self._store)))
            self._evictions += 1

    def _result(self, entry: CacheEntry) -> CacheLookupResult:
        dev, conf = entry.predict_device()
        low = conf < self.prediction_confidence_threshold
        if low:
            self._hybrid_fallbacks += 1
        return CacheLookupResult(entry, dev, conf, low)

    # ------------------------------------------------------------------ API
    def lookup(self, query: str, context_key: str, q_emb: Any = None) -> Optional[CacheLookupResult]:
        with self._lock:
            self._attempts += 1
        self._evict_expired()
        h = self._make_hash(query, context_key)
        with self._lock:
            pre = self._pre.pop((query, context_key), None) if self._pre else None
            if not self._pre:   # the batch is consumed: stop tracking changed contexts
                self._index.track_dirty = False
            cand = self._store.get(h)
            if cand is not None and cand.context_key == context_key:
                if self._is_valid(cand):
                    cand.hit_count += 1
                    self._store.move_to_end(h)
                    self._hits += 1
                    return self._result(cand)
                self._delete_entry(h)
            if not self.use_semantic or q_emb is None:
                return None
            cid = self._index.cid_of(context_key)
            if pre is not None and (cid is None or cid not in self._index.dirty):
                slot = pre[0]           # no row of this context changed since the batch was scored
                self.prefetch_used += 1
            else:
                if pre is not None:
                    self.prefetch_fallbacks += 1
                slot, _sim = self._index.best(q_emb, context_key, self.similarity_threshold)
            if slot < 0:
                return None
            bh = self._slot_to_hash.get(slot)
            cand = self._store.get(bh) if bh else None
            if cand is None or not self._is_valid(cand):
                return None
            cand.hit_count += 1
            self._store.move_to_end(bh)
            self._hits += 1
            return self._result(cand)

    def prefetch(self, items: List[Tuple[str, str, Any]]) -> None:
        """Score the semantic lookups of a whole routing batch at once: ``items`` = (query,
        context_key, q_emb) in the order the batch will be routed.  On an HBM index this is one
        launch and one read-back for the batch instead of one of each per lookup.  ``lookup``
        then uses a query's prefetched result only while no row of its context has changed since
        (an insert, replacement, TTL or LRU eviction in between marks the context dirty and that
        lookup is re-scored on its own), so routing decisions are exactly those of per-query
        lookups."""
        if not self.use_semantic:
            return
        self._evict_expired()
        with self._lock:
            self._pre = {}
            self._index.dirty.clear()
            self._index.track_dirty = False
            items = [(q, ck, e) for q, ck, e in items if e is not None]
            if not items:
                return
            self._index.track_dirty = True
            res = self._index.best_batch([e for _, _, e in items], [ck for _, ck, _ in items],
                                         self.similarity_threshold)
            for (q, ck, _), r in zip(items, res):
                self._pre[(q, ck)] = r

    def insert(self, query: str, context_key: str, device: str, confidence: float = 1.0,
               method: str = "unknown", q_emb: Any = None, response_time: Optional[float] = None) -> None:
        h = self._make_hash(query, context_key)
        with self._lock:
            e = self._store.get(h)
            if e is not None:
                self._stamp(e)
                e.record_routing(device, confidence, method)
                self._set_embedding(e, q_emb)
                if response_time is not None:
                    e.response_time = response_time
                self._store.move_to_end(h)
                return
            if len(self._store) >= self.max_size:
                self._evict_one()
            e = CacheEntry(query=query, query_hash=h, context_key=context_key, embedding=None,
                           timestamp=datetime.now(), device_used=device, response_time=response_time)
            self._stamp(e, e.timestamp)
            self._set_embedding(e, q_emb)
            e.record_routing(device, confidence, method)
            self._store[h] = e

    def invalidate(self, context_key: Optional[str] = None, query_pattern: Optional[str] = None) -> int:
        pat = re.compile(query_pattern, re.IGNORECASE) if query_pattern else None
        with self._lock:
            doomed = [h for h, e in self._store.items()
                      if (context_key is None or e.context_key == context_key)
                      and (pat is None or pat.search(e.query))]
            for h in doomed:
                self._delete_entry(h)
        return len(doomed)

    def warm_up(self, pairs: List[Tuple[str, str, str]], embedder: Any = None) -> None:
        vecs: List[Optional[np.ndarray]] = [None] * len(pairs)
        if embedder is not None and pairs:
            try:
                vecs = list(embedder.encode([q for q, _, _ in pairs]))
            except Exception as exc:  # embedding is optional for warm-up
                logger.warning("warm_up: embedding failed, skipping vectors: %s", exc)
        for (q, ck, dev), v in zip(pairs, vecs):
            self.insert(q, ck, dev, q_emb=v)

    def save(self, path: str) -> None:
        """Reference JSON format (`src/cache.py:426-432`); a ``.safetensors`` path writes the
        binary snapshot instead (see :meth:`save_snapshot`)."""
        if str(path).endswith(".safetensors"):
            self.save_snapshot(path)
            return
        self._evict_expired()
        with self._lock:
            data = [e.to_dict() for e in self._store.values()]
        Path(path).write_text(json.dumps(data, indent=2), encoding="utf-8")

    def load(self, path: str) -> int:
        if str(path).endswith(".safetensors"):
            return self.load_snapshot(path)
        p = Path(path)
        if not p.exists():
            return 0
        try:
            raw = json.loads(p.read_text(encoding="utf-8"))
        except json.JSONDecodeError as exc:
            logger.error("Cache load: JSON parse error: %s", exc)
            return 0
        return self._ingest((d, None) for d in raw)

    def _ingest(self, items) -> int:
        """Insert (entry dict, optional embedding override) pairs; skips expired / malformed."""
        n = 0
        with self._lock:
            for d, emb_override in items:
                try:
                    e = CacheEntry.from_dict(d)
                except Exception as exc:
                    logger.warning("Cache load: skipping malformed entry: %s", exc)
                    continue
                if not self._is_valid(e):
                    continue
                if e.query_hash in self._store:
                    self._delete_entry(e.query_hash)
                emb, e.embedding = (emb_override if emb_override is not None else e.embedding), None
                self._set_embedding(e, emb)
                self._store[e.query_hash] = e
                self._stamp(e, e.timestamp)
                n += 1
        return n

    def save_snapshot(self, path: str) -> None:
        """Binary snapshot: the embedding table as one f32 [n, dim] safetensors
        tensor plus the entries (without vectors) as JSON in the file's metadata. A million-entry
        cache is ~1.5 GB of raw f32 instead of ~8 GB of JSON float text, and loads with one read."""
        from safetensors.numpy import save_file
        self._evict_expired()
        with self._lock:
            entries = list(self._store.values())
            metas, rows = [], []
            for e in entries:
                d = e.to_dict()
                d["embedding"] = None
                d["emb_row"] = len(rows) if e.embedding is not None else -1
                if e.embedding is not None:
                    rows.append(_host_vec(e.embedding))
                metas.append(d)
        dim = rows[0].shape[0] if rows else self._index.dim
        table = np.stack(rows) if rows else np.zeros((0, dim), dtype=np.float32)
        save_file({"embeddings": np.ascontiguousarray(table)}, str(path),
                  metadata={"format": "dllm-routing-cache-v1", "entries": json.dumps(metas)})

    def load_snapshot(self, path: str) -> int:
        from safetensors import safe_open
        p = Path(path)
        if not p.exists():
            return 0
        try:
            with safe_open(str(p), framework="numpy") as f:
                meta = f.metadata() or {}
                table = f.get_tensor("embeddings")
        except Exception as exc:
            logger.error("Cache snapshot load failed: %s", exc)
            return 0
        if meta.get("format") != "dllm-routing-cache-v1":
            logger.error("Cache snapshot load: unknown format %r", meta.get("format"))
            return 0
        metas = json.loads(meta.get("entries", "[]"))

        def items():
            for d in metas:
                r = int(d.pop("emb_row", -1))
                yield d, (table[r] if 0 <= r < table.shape[0] else None)
        return self._ingest(items())

    def stats(self) -> Dict[str, Any]:
        with self._lock:
            now = datetime.now()
            valid = sum(1 for e in self._store.values() if self._is_valid(e, now))
            size = len(self._store)
            hot = sorted(self._store.values(), key=lambda e: e.hit_count, reverse=True)[:5]
            top = []
            for e in hot:
                dev, conf = e.predict_device()
                top.append({"query": e.query[:60], "hits": e.hit_count, "predicted_device": dev,
                            "predicted_confidence": round(conf, 3),
                            "history_len": len(e.routing_history)})
            return {"size": size, "max_size": self.max_size, "valid": valid, "stale": size - valid,
                    "hits": self._hits, "attempts": self._attempts,
                    "hit_rate": round(self._hits / max(self._attempts, 1), 4),
                    "evictions": self._evictions, "hybrid_fallbacks": self._hybrid_fallbacks,
                    "top_queries": top}

    def clear(self) -> None:
        with self._lock:
            self._store.clear()
            self._slot_to_hash.clear()
            self._index.clear()
            self._expiry.clear()
            self._pre = {}
            self._hits = self._attempts = self._evictions = self._hybrid_fallbacks = 0

    def __len__(self) -> int:
        return len(self._store)
