#!/usr/bin/env python3
"""Flagship benchmark: routed end-to-end serving on MI355X (BASELINE.json metric).

Reference workload (src/tests/routing_chatbot_tester.py:405-486): each query set is replayed as
ONE growing conversation; every turn is routed (token / heuristic / semantic / hybrid / perf) to
the small or large tier and answered there; latency and response tokens are recorded per turn.

One GPU (the default, ``--topology replicated``): BASELINE config 2 — TinyLlama-1.1B architecture
(random-init bf16 weights, fixed seed: no checkpoints exist in this environment) serving BOTH tiers
from one engine, hybrid router with the semantic routing cache on (HBM-resident cache table, GPU
MiniLM-L6 encoder).  The GPU serves ``--convs`` concurrent conversations (the three reference
query sets round-robin, each conversation tagged with a unique session so no two share KV prefixes
or answers).  One *step* = one turn of every conversation: route all, then the engine serves the
small- and large-tier groups as one continuous batch (paged KV, prefix cache across turns, hipGraph
decode).  The response cache is OFF (its context-free key would replay other conversations'
answers = skipped work); small tier greedy (reference Nano), large tier Ollama-default sampling
(reference Orin).  By default the conversations are turn-PIPELINED (``--pipeline 2``): one driver
thread routes every conversation whose answer has arrived and submits its next turn without
waiting for the others (each conversation stays strictly sequential, as in the reference harness),
so the decode batch stays full instead of draining to the large-tier answers at the end of every
turn; a *step* is then ``--convs`` completed turns, and only turns completed inside the timed
window are counted.  ``--pipeline 0`` runs the turn-synchronous steps of rounds 1-3.

N > 1 GPUs run N config-2 replicas by default (``--topology replicated``: one engine and one routing
driver per GPU, each with its own --convs conversations; per-GPU work is fixed, so values at N = 1, 2, 4, 8 form a weak-scaling
curve of ONE workload).  BASELINE's multi-GPU configurations are selected with ``--baseline-config``
(or ``--topology pools``, parallel.cluster):
2 GPUs config 3 (Llama-3.2-1B small on GPU 0 | Llama-3-8B large on GPU 1), 4 GPUs config 4's models
at half size (Llama-3-8B x2 | Llama-3-70B TP=2), 8 GPUs config 4 (Llama-3-8B x4 | Llama-3-70B
TP=4, perf router), and ``--baseline-config 5`` (``--topology colocated``) config 5 as written:
Mixtral-8x7B TP=N over every GPU with a Llama-3.2-1B small replica co-located on each GPU.  Rank 0
hosts the router and drives ``--convs x N`` conversations (``--convs`` defaults to 128 per GPU
there: with the event driver serving remote pools non-blockingly, 128 per GPU gave 17.3k vs 11.4k
routed tok/s at 64 on the 2-rank config-3 rehearsal, while an 8B-tier GPU's 64 GB KV pool still
holds 128 conversations at ~3K tokens of history each); requests reach remote pools over the gloo control / data planes, RCCL carries the large
pool's tensor-parallel collectives.  The JSON line names the config (``baseline_config``) and the
exact GPU layout (``layout``); values of different configs are different model configurations,
not a scaling curve (``scaling_note``).

``value`` = total generated tokens over all ranks / max rank wall time of the timed steps.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import queue
import statistics
import sys
import time

from distributed_llm_amd.utils.faults import diag

_T_PROC0 = time.perf_counter()   # process start (imports included) for the JSON's startup_s

BASELINE_TOK_S = 10.57        # best published routed throughput (Jetson Nano+Orin)
BASELINE_S_PER_QUERY = 39.6   # best published mean routed e2e latency per query


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--topology", default=None, choices=["replicated", "pools", "colocated", "tiers"],
                    help="replicated: both tiers on one engine per GPU (BASELINE config 2; the 1-GPU default); "
                         "pools: tiers on disjoint GPU subsets (configs 3-4); colocated: large "
                         "TP group over every GPU + a small replica on each GPU (config 5); tiers: --small-model "
                         "and --large-model as two engines on every GPU")
    ap.add_argument("--baseline-config", type=int, default=None, choices=[2, 3, 4, 5],
                    help="BASELINE.json config to run (default 2 at every N; 3 needs 2 GPUs, 4 needs 4-8); "
                         "sets topology and models")
    ap.add_argument("--model", default="tinyllama-1.1b")
    ap.add_argument("--small-model", default=None, help="pools/tiers small tier (default per baseline config)")
    ap.add_argument("--large-model", default=None, help="pools/tiers large tier (default per baseline config)")
    ap.add_argument("--large-tp", type=int, default=None)
    ap.add_argument("--layers", type=int, default=None,
                    help="truncate every model to its first N decoder layers (rehearsals of the big configs on "
                         "one GPU; the JSON line says so); never for a reported number")
    ap.add_argument("--convs", type=int, default=None,
                    help="concurrent conversations per GPU (default 512; 64 for the multi-GPU pool configs)")
    ap.add_argument("--strategy", default=None, help="routing strategy (default: perf for config 4, else hybrid)")
    ap.add_argument("--threshold", type=int, default=1000)
    ap.add_argument("--small-new", type=int, default=128)
    ap.add_argument("--large-new", type=int, default=384)
    ap.add_argument("--kv-gb", type=float, default=None,
                    help="KV cache per engine (GB); default 64, or 160 for a pool engine that owns its GPU "
                         "(pools topology, N > 1: 128 conversations per GPU at ~3K tokens of history)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--cpu", action="store_true", help="CPU plumbing run (tiny model)")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="turn pipelining: conversations advance independently; 0: turn-synchronous steps, "
                         "1: one thread per conversation, 2: one event-driven driver thread (the default, every "
                         "topology: +6-7 %% routed tok/s on one GPU, decode batch 372 -> 495-500 of 512, "
                         "profiles/r4_turn_pipelining.md)")
    ap.add_argument("--gil-switch-ms", type=float, default=0.5,
                    help="turn pipelining: Python thread switch interval (sys.setswitchinterval) in ms")
    ap.add_argument("--admit-every", type=int, default=16,
                    help="turn pipelining: the engine admits new turns every N decode steps of a burst")
    ap.add_argument("--no-encoder-memo", action="store_true",
                    help="encode every routed query with the GPU MiniLM encoder (no per-text memo)")
    ap.add_argument("--greedy", action="store_true",
                    help="both tiers greedy (the large tier samples top-k 40 / top-p 0.9 at T 0.8 otherwise); "
                         "for token-exact cross-topology checks")
    ap.add_argument("--dump-responses", default=None,
                    help="rank 0 writes every timed turn's (conversation, turn, tier, response text) as JSON here")
    ap.add_argument("--trace", default=None,
                    help="write a Chrome trace (router/pool/engine spans, GPU decode time) to this path; "
                         "'{rank}' is replaced by the rank")
    return ap.parse_args()


# BASELINE.json "configs" (1-based) -> (topology, small model, large model, large TP or None = default)
BASELINE_CONFIGS = {
    2: ("replicated", None, None, None),
    3: ("pools", "llama-3.2-1b", "llama-3-8b", None),         # 1B | 8B, one GPU each (2 GPUs)
    4: ("pools", "llama-3-8b", "llama-3-70b", 4),             # 8B replicas | 70B TP=4 over xGMI
    5: ("colocated", "llama-3.2-1b", "mixtral-8x7b", None),   # Mixtral TP=N + a 1B replica on every GPU
}


def resolve_config(a, world: int) -> int:
    """Fill topology / models from ``--baseline-config`` (or infer it) and return the config id
    tagged on the JSON line."""
    cfg = a.baseline_config
    if a.topology is None and cfg is None:
        # every N defaults to config 2 (one engine per GPU): the driver's N = 1 .. 8 runs are then
        # one workload's weak-scaling curve; the multi-GPU configs 3-5 are --baseline-config runs
        a.topology = "replicated"
    if cfg is None:
        if a.topology == "colocated":
            cfg = 5
        elif a.topology == "pools" and world > 1:
            cfg = 4 if world >= 4 else 3
        else:
            cfg = 2
    topo, sm, lg, tp = BASELINE_CONFIGS[cfg]
    if a.baseline_config is not None or a.topology is None:
        a.topology = topo
    if a.convs is None:
        a.convs = 128 if (world > 1 and a.topology in ("pools", "colocated")) else 512
    a.small_model = a.small_model or sm or "llama-3.2-1b"
    a.large_model = a.large_model or lg or "llama-3-8b"
    if a.large_tp is None and tp is not None and world >= 2 * tp:
        a.large_tp = tp
    a.strategy = a.strategy or ("perf" if cfg == 4 else "hybrid")   # config 4: perf-router failover
    return cfg


def _router_stream() -> None:
    """Pipelined drivers route while the engine's loop keeps decode steps queued on its stream:
    the router's own GPU work (encoder, centroid scores, HBM cache lookups, each read back to the
    host) goes to a side stream of this thread, so its read-backs wait for the router's kernels
    only, not for the decode step queued ahead of them on the engine's stream."""
    import torch
    global _ROUTER_STREAM
    if torch.cuda.is_available():
        if _ROUTER_STREAM is None:
            _ROUTER_STREAM = torch.cuda.Stream()   # one for every driver thread of the process
        torch.cuda.set_stream(_ROUTER_STREAM)


_ROUTER_STREAM = None


class Conversations:
    def __init__(self, n: int, rank: int):
        from distributed_llm_amd.bench.query_sets import normalize_query_set, query_sets
        self.sets = [normalize_query_set(query_sets[k]) for k in ("general_knowledge", "technical_coding",
                                                                  "personal_health")]
        self.rank, self._ids = rank, itertools.count(1)   # next() is atomic: safe from worker threads
        self.convs = [self._new(i) for i in range(n)]
        self.steps_done = 0

    def _new(self, i):
        return {"set": self.sets[i % 3], "turn": 0, "hist": [], "tag": f"[session r{self.rank}-{next(self._ids)}] "}

    def step(self, router, records=None, dump=None):
        hs = []
        for c in self.convs:
            q = c["set"][c["turn"]].text
            if c["turn"] == 0:
                q = c["tag"] + q
            c["hist"].append({"role": "user", "content": q})
            hs.append(c["hist"])
        t0 = time.perf_counter()
        res = router.route_batch(hs)
        lat = (time.perf_counter() - t0) * 1000.0   # client side: every turn of the step waits for the batch
        for i, (c, (payload, ntok, device)) in enumerate(zip(self.convs, res)):
            c["hist"].append({"role": "assistant", "content": payload["response"]})
            if dump is not None:
                dump.append([i, c["turn"], device, payload["response"]])
            if records is not None:
                raw = payload.get("raw") or {}
                records.append({"lat": lat,
                                "lat_engine": float(raw.get("latency_ms", 0.0)) if isinstance(raw, dict) else 0.0,
                                "tok": int(ntok), "dev": device, "fo": payload.get("failover_from"),
                                "ok": bool(payload.get("ok", True)), "step": self.steps_done,
                                "ovh": float(payload.get("routing_overhead_ms", 0.0)),
                                "ttft": float(((raw.get("timing") or {}) if isinstance(raw, dict) else {})
                                              .get("ttft_ms", 0.0))})
            c["turn"] += 1
            if c["turn"] >= len(c["set"]):
                self.convs[i] = self._new(i)
        self.steps_done += 1


class PipelinedConversations(Conversations):
    """Turn pipelining: one thread per conversation runs route -> serve -> next turn on its own.

    Each conversation stays strictly sequential (turn t+1 is built from turn t's answer, as in
    the reference harness, routing_chatbot_tester.py:405-486), but conversations no longer wait
    for each other: a conversation whose small-tier answer (<= 128 tokens) is done submits its
    next turn while large-tier answers (<= 384 tokens) are still decoding, so the engine's decode
    batch stays full instead of draining to the large-tier share at the end of every step.

    Steady-state accounting: with no per-step barrier a *step* is ``n_convs`` completed turns
    (one turn per conversation on average).  ``start()`` launches the workers; ``wait_turns(n)``
    blocks until ``n`` turns in total have completed.  Only turns that complete inside the timed
    window are recorded and counted (a turn in flight at the window's end is not counted; one in
    flight at its start is counted whole), so no work is skipped or double counted."""

    def start(self, router) -> None:
        import threading
        self._cv = threading.Condition()
        self.completed = 0
        self.records = None
        self._stop = False
        self.errors = []

        def worker(i):
            try:
                _router_stream()
                while not self._stop:
                    c = self.convs[i]
                    q = c["set"][c["turn"]].text
                    if c["turn"] == 0:
                        q = c["tag"] + q
                    c["hist"].append({"role": "user", "content": q})
                    t0 = time.perf_counter()
                    payload, ntok, device = router.route_concurrent(c["hist"])
                    lat = (time.perf_counter() - t0) * 1000.0
                    c["hist"].append({"role": "assistant", "content": payload["response"]})
                    raw = payload.get("raw") if isinstance(payload.get("raw"), dict) else {}
                    rec = {"lat": lat, "lat_engine": float(raw.get("latency_ms", 0.0)), "tok": int(ntok), "dev": device,
                           "ovh": float(payload.get("routing_overhead_ms", 0.0)),
                           "ttft": float((raw.get("timing") or {}).get("ttft_ms", 0.0))}
                    c["turn"] += 1
                    if c["turn"] >= len(c["set"]):
                        self.convs[i] = self._new(i)
                    with self._cv:
                        if self.records is not None:
                            self.records.append(rec)
                        self.completed += 1
                        self._cv.notify_all()
            except BaseException as e:  # surfaced by wait_turns
                with self._cv:
                    self.errors.append(e)
                    self._cv.notify_all()

        self._threads = [threading.Thread(target=worker, args=(i,), daemon=True) for i in range(len(self.convs))]
        for t in self._threads:
            t.start()

    def wait_turns(self, n: int, records=None) -> None:
        """Block until ``n`` turns have completed in total; from then on record into ``records``."""
        # DLLM_VERBOSE=1: a progress line every 30 s (long rehearsals; gpurun's silence watchdog)
        verbose = os.environ.get("DLLM_VERBOSE") == "1"
        last = time.perf_counter()
        with self._cv:
            while self.completed < n and not self.errors:
                self._cv.wait(timeout=30.0 if verbose else None)
                if verbose and time.perf_counter() - last >= 30.0:
                    last = time.perf_counter()
                    print(f"bench: {self.completed} / {n} turns completed", file=sys.stderr, flush=True)
            if self.errors:
                raise self.errors[0]
            self.records = records

    def stop(self) -> None:
        self._stop = True            # workers exit after their in-flight turn
        for t in self._threads:
            t.join()


def _thread_cpu() -> dict:
    """CPU seconds per named Python thread of this process (``DLLM_DIAG=cpu`` diagnostics:
    how much of the window the routing driver and each engine's step loop hold a core / the GIL)."""
    import threading
    import psutil
    names = {t.native_id: t.name for t in threading.enumerate()}
    out = {}
    for th in psutil.Process().threads():
        k = names.get(th.id, "other")
        out[k] = out.get(k, 0.0) + th.user_time + th.system_time
    return out


class EventConversations(PipelinedConversations):
    """Turn pipelining from ONE driver thread (``--pipeline 2``): every conversation whose answer
    has arrived is routed (one batched decision pass for all of them, ``Router.dispatch_batch``)
    and its next turn is submitted to the engine without blocking; the driver then blocks on a
    completion queue the engines feed (``notify``) and collects whatever finished -- no polling
    of in-flight handles (at 512 conversations that scan cost the driver ~0.1 of a core in GIL
    holds, profiles/r4_host_cpu_budget.md).  Each conversation stays strictly sequential, the continuous
    batch stays full (a small-tier answer's conversation re-enters while large-tier answers are
    still decoding), and there is no per-conversation thread competing for the GIL.  The engine
    admits new turns every ``--admit-every`` decode steps so its pipelined bursts stay long.
    Same steady-state window accounting as the parent (a step = ``n_convs`` completed turns)."""

    WAIT_S = 0.05     # longest block on the completion queue (re-checks the stop flag)

    def start(self, router) -> None:
        import threading
        self._cv = threading.Condition()
        self.completed = 0
        self.records = None
        self._stop = False
        self.errors = []

        def driver():
            prof = None
            if diag("profile"):   # cProfile of this thread, dumped at stop() (DLLM_DIAG=profile=PATH)
                import cProfile
                prof = cProfile.Profile()
                prof.enable()
            try:
                _router_stream()
                ready = list(range(len(self.convs)))
                inflight = {}          # id(handle) -> (conversation, ticket); handle-less: own key
                keys = {}              # conversation -> its in-flight ticket's key
                finished = queue.SimpleQueue()   # handles the pools finished (notify)

                def track(i, t):
                    h = t.get("handle")
                    keys[i] = id(h) if h is not None else ("t", i)
                    inflight[keys[i]] = (i, t)
                    return router.ticket_done(t)   # cache hit, served inline, rejected, or already finished

                again = []             # failed-over tickets already done when re-submitted
                while not self._stop:
                    done, again = again, []
                    if ready:
                        hs = []
                        for i in ready:
                            c = self.convs[i]
                            q = c["set"][c["turn"]].text
                            if c["turn"] == 0:
                                q = c["tag"] + q
                            c["hist"].append({"role": "user", "content": q})
                            hs.append(c["hist"])
                        for i, t in zip(ready, router.dispatch_batch(hs, notify=finished.put)):
                            if track(i, t):
                                done.append(i)
                        ready = []
                    # block on the pools' completion queue instead of scanning every ticket
                    items = []
                    try:
                        if not done:
                            items.append(finished.get(timeout=self.WAIT_S))
                        while True:
                            items.append(finished.get_nowait())
                    except queue.Empty:
                        pass
                    for h in items:
                        e = inflight.get(id(h))
                        if e is not None and e[1].get("handle") is h:
                            done.append(e[0])
                    if not done:
                        continue
                    tickets = {}       # a ticket can be both notified and seen done on dispatch
                    for i in done:
                        if i not in tickets and i in keys:
                            tickets[i] = inflight.pop(keys.pop(i))[1]
                    recs = []
                    for i, t in tickets.items():
                        res = router.finish_ticket(t, notify=finished.put)
                        if res is None:              # failed over: in flight on the other tier
                            if track(i, t):
                                again.append(i)
                            continue
                        payload, ntok, device = res
                        c = self.convs[i]
                        c["hist"].append({"role": "assistant", "content": payload["response"]})
                        raw = payload.get("raw") if isinstance(payload.get("raw"), dict) else {}
                        recs.append({"lat": float(t.get("latency_ms", 0.0)),
                                     "lat_engine": float(raw.get("latency_ms", 0.0)), "tok": int(ntok),
                                     "dev": device, "ovh": float(payload.get("routing_overhead_ms", 0.0)),
                                     "ttft": float((raw.get("timing") or {}).get("ttft_ms", 0.0)),
                                     "fo": payload.get("failover_from"), "ok": bool(payload.get("ok", True)),
                                     "step": self.completed // max(1, len(self.convs))})
                        c["turn"] += 1
                        if c["turn"] >= len(c["set"]):
                            self.convs[i] = self._new(i)
                        ready.append(i)
                    with self._cv:
                        if self.records is not None:
                            self.records.extend(recs)
                        self.completed += len(recs)
                        self._cv.notify_all()
            except BaseException as e:  # surfaced by wait_turns
                with self._cv:
                    self.errors.append(e)
                    self._cv.notify_all()
            finally:
                if prof is not None:
                    prof.disable()
                    prof.dump_stats(diag("profile"))

        self._threads = [threading.Thread(target=driver, name="bench-driver", daemon=True)]
        self._threads[0].start()


STEP_LOOP_TIMERS = ("t_prefill_s", "t_admit_s", "t_decode_host_pre_s", "t_decode_gpu_wait_s",
                    "t_decode_host_post_s", "t_complete_s")
CLIENT_TIMERS = ("t_encode_s", "t_output_s")


def _collective_cross_check(tokens, elapsed, dev, world):
    """(backend, tokens summed, window max) from two all-reduces on ``dev`` (RCCL on a GPU node, gloo
    on CPU); None if they did not finish within 60 s."""
    import datetime
    import torch
    import torch.distributed as dist
    try:
        s_t = torch.tensor([float(tokens)], dtype=torch.float64, device=dev)
        m_t = torch.tensor([float(elapsed)], dtype=torch.float64, device=dev)
        w1 = dist.all_reduce(s_t, op=dist.ReduceOp.SUM, async_op=True)
        w2 = dist.all_reduce(m_t, op=dist.ReduceOp.MAX, async_op=True)
        w1.wait(timeout=datetime.timedelta(seconds=60))
        w2.wait(timeout=datetime.timedelta(seconds=60))
        if s_t.is_cuda:
            torch.cuda.synchronize()
        return {"backend": str(dist.get_backend()), "ranks": world, "tokens_sum": s_t.item(),
                "elapsed_max_s": m_t.item()}
    except Exception as e:  # noqa: BLE001 - reported, never fatal: the store reduction is authoritative
        return {"backend": str(dist.get_backend()), "error": repr(e)[:200]}


def _peak_mem_gb(on_gpu: bool):
    """This process's peak PyTorch device allocation (weights, KV pool, workspaces, graphs), GB."""
    if not on_gpu:
        return None
    import torch
    return round(torch.cuda.max_memory_allocated() / 2**30, 2)


def kv_placement(st0, st1):
    d = lambda k: sum(b.get(k, 0) - a_.get(k, 0) for a_, b in zip(st0, st1))
    run, seg, tot = d("contiguous_allocs"), d("segment_allocs"), d("fresh_allocs")
    # every new block either continues its sequence's run, opens a wholly free segment, or comes
    # from the free list / LRU (scattered)
    out = {"new_blocks": int(tot), "run_share": round(run / tot, 3) if tot else None,
           "segment_share": round(seg / tot, 3) if tot else None}
    # why the others did not continue: no previous block (a sequence's first), next block held by a
    # live sequence, next block cached but hot (block_manager.h fresh)
    for k in ("roomy_segment_allocs", "inplace_evictions", "run_miss_first", "run_miss_held", "run_miss_hot",
              "run_miss_held_shared", "run_miss_held_segstart"):
        out[k.replace("_allocs", "").replace("_evictions", "") + "_share"] = round(d(k) / tot, 3) if tot else None
    roomy = d("roomy_segment_allocs")
    out["roomy_stretch_mean_blocks"] = round(d("roomy_stretch_blocks") / roomy, 1) if roomy else None
    return out


def engine_time_split(st0, st1, window_s: float) -> dict:
    """Where the timed window went, per THREAD.  The step-loop timers are disjoint, so with one engine
    they partition its thread's window (``step_loop_other_s``: waiting for work, scheduling glue);
    the caller-side timers (prompt encode at submit, results) run on the routing threads at the same
    time and are reported apart, never subtracted from the window (which made the round-4 field
    negative).  Several engines (co-located tiers, replicas) each have their own step loop: their
    sums are reported without the remainder."""
    d = lambda k: round(sum(b.get(k, 0.0) - a.get(k, 0.0) for a, b in zip(st0, st1)), 3)
    loop = {k: d(k) for k in STEP_LOOP_TIMERS}
    if len(st0) == 1:
        loop["step_loop_other_s"] = round(max(0.0, window_s - sum(loop.values())), 3)
    return {"step_loop": loop, "caller_threads": {k: d(k) for k in CLIENT_TIMERS}, "engines": len(st0)}


def main() -> int:
    a = parse()
    if os.environ.get("DLLM_STACK_DUMP_S"):   # diagnostics: every thread's stack after S seconds (hang hunting)
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["DLLM_STACK_DUMP_S"]), exit=False)
    import torch
    import torch.distributed as dist
    from distributed_llm_amd.config import LARGE, PRODUCTION_CFG, SMALL
    from distributed_llm_amd.orchestrator import Router

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if a.trace:
        from distributed_llm_amd.utils.tracing import tracer
        tracer.enable(a.trace.replace("{rank}", str(rank)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    on_gpu = torch.cuda.is_available() and not a.cpu
    # DLLM_REHEARSE_ONE_GPU=1: every rank on GPU 0 with gloo collectives — rehearses the N-rank
    # bench path (process group, per-rank engines and graphs, barriers, cross-rank reduction) on a
    # one-GPU box; RCCL itself refuses two ranks on one device.  Never used for reported numbers.
    rehearse = world > 1 and on_gpu and os.environ.get("DLLM_REHEARSE_ONE_GPU") == "1"
    kv_gb = a.kv_gb if a.kv_gb is not None else 64.0
    if rehearse:
        local = 0
    coll_dev = "cpu" if (rehearse or not on_gpu) else f"cuda:{local}"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if on_gpu:
            torch.cuda.set_device(local)
        dist.init_process_group("nccl" if on_gpu and not rehearse else "gloo")
    dev = f"cuda:{local}" if on_gpu else "cpu"
    if not on_gpu:
        os.environ.setdefault("DLLM_EMBEDDER", "hash")
    if a.no_encoder_memo:
        os.environ["DLLM_ENCODER_MEMO"] = "0"
    from distributed_llm_amd.router.embedder import encoder_stats
    baseline_config = resolve_config(a, world)
    topology = a.topology if (world > 1 or a.topology == "tiers") else "replicated"
    if topology == "replicated":
        baseline_config = 2
    layout = None
    cfg = dict(PRODUCTION_CFG, token_threshold=a.threshold, enable_response_cache=False, tokens_from_engine=True,
               cache_index_device=dev if on_gpu else None, cache_max_size=1 << 20)
    if topology in ("pools", "colocated"):
        # the multi-GPU configs are failover tests too (config 4: "perf-router failover"): a failed
        # tier is charged in the perf router, which also tries an unseen tier
        cfg.update(penalise_failed_primary=True, perf_explore=True)

    # reference Orin defaults (Ollama: T 0.8, top-k 40, top-p 0.9); --greedy for exact comparisons
    large_sampling = (dict(temperature=0.0, top_k=0, top_p=1.0) if a.greedy
                      else dict(temperature=0.8, top_k=40, top_p=0.9))
    cluster = None

    def mdl(name):
        """A model to build: the registry name, or its layer-truncated config under --layers."""
        if not a.layers:
            return name
        from distributed_llm_amd.models.configs import get_model_config
        return get_model_config(name, n_layers=a.layers)

    if topology == "tiers":
        # heterogeneous tiers co-located on each GPU: a small-model engine and a large-model engine
        # (BASELINE config 3's model pair; the reference runs them on two boards)
        from distributed_llm_amd.engine.llm_engine import LLMEngine
        from distributed_llm_amd.pools.base import EnginePool
        sm = a.small_model if on_gpu else "tiny-llama-test"
        lg = a.large_model if on_gpu else "tiny-llama-test"
        kv = (kv_gb / 2) if on_gpu else 0.1
        e_small = LLMEngine(mdl(sm), device=dev, kv_cache_gb=kv, max_num_seqs=max(16, a.convs),
                            use_graphs=not a.no_graphs, seed=0)
        e_large = LLMEngine(mdl(lg), device=dev, kv_cache_gb=kv, max_num_seqs=max(16, a.convs),
                            use_graphs=not a.no_graphs, seed=0)   # seed 0 like the pools' engines
        pools = {SMALL: EnginePool(SMALL, e_small, max_new_tokens=a.small_new, temperature=0.0),
                 LARGE: EnginePool(LARGE, e_large, max_new_tokens=a.large_new, **large_sampling)}
        if on_gpu:
            for e in (e_small, e_large):
                e.capture_all(max_bs=e._bucket(max(16, a.convs)))
        engines = [e_small, e_large]
        model_desc = f"{sm} small + {lg} large (two engines co-located per GPU)"
        n_convs, parallelism = a.convs, f"dp{world}-colocated-tiers"
        layout = {"small": {"model": sm, "replicas": [[r] for r in range(world)], "tp": 1},
                  "large": {"model": lg, "replicas": [[r] for r in range(world)], "tp": 1}, "colocated": True}
    elif topology == "replicated":
        from distributed_llm_amd.engine.llm_engine import LLMEngine
        from distributed_llm_amd.pools.base import EnginePool
        model = a.model if on_gpu else "tiny-llama-test"
        engine = LLMEngine(mdl(model), device=dev, kv_cache_gb=kv_gb if on_gpu else 0.2,
                           max_num_seqs=max(16, a.convs), use_graphs=not a.no_graphs, seed=0)
        pools = {SMALL: EnginePool(SMALL, engine, max_new_tokens=a.small_new, temperature=0.0),
                 LARGE: EnginePool(LARGE, engine, max_new_tokens=a.large_new, **large_sampling)}
        if on_gpu:
            engine.capture_all(max_bs=engine._bucket(max(16, a.convs)))
        engines = [engine]
        model_desc = f"{model} (small+large tiers on one engine per GPU)" if on_gpu else model
        n_convs, parallelism = a.convs, f"dp{world}"
        layout = {"small": {"model": model, "replicas": [[r] for r in range(world)], "tp": 1},
                  "large": {"model": model, "replicas": [[r] for r in range(world)], "tp": 1,
                            "shared_engine_with_small": True}}
    else:
        from distributed_llm_amd.parallel.cluster import Cluster, TierSpec, default_topology
        topo = default_topology(world, a.large_tp, colocated=(topology == "colocated"))
        sm = a.small_model if on_gpu else "tiny-llama-test"
        lg = a.large_model if on_gpu else "tiny-moe-test"
        n_small = len(topo.replicas[SMALL])
        # (a one-GPU rehearsal runs the TP collectives on gloo, which a hipGraph cannot capture; tiers
        # without TP groups capture their decode graphs as on a real node)
        graphs = {t: not (a.no_graphs or (rehearse and max(len(g) for g in topo.replicas[t]) > 1))
                  for t in (SMALL, LARGE)}
        # a pool engine that owns its GPU (disjoint pools on a real node) gets a larger KV pool: the
        # Llama-3-8B small replicas of config 4 hold 128 conversations x ~3K tokens x 128 KB
        if a.kv_gb is None and topology == "pools" and not rehearse:
            kv_gb = 160.0
        specs = {SMALL: TierSpec(mdl(sm), a.small_new, 0.0, kv_cache_gb=kv_gb if on_gpu else 0.1,
                                 max_num_seqs=max(16, a.convs * world), graphs=graphs[SMALL]),
                 LARGE: TierSpec(mdl(lg), a.large_new, large_sampling["temperature"], large_sampling["top_k"],
                                 large_sampling["top_p"], kv_cache_gb=kv_gb if on_gpu else 0.1,
                                 max_num_seqs=max(16, a.convs * world), graphs=graphs[LARGE])}
        cluster = Cluster(topo, specs, device=dev)
        engines = list(cluster.engines.values())
        if on_gpu:
            for e in engines:
                if e.use_graphs:
                    e.capture_all(max_bs=e._bucket(min(e.R, max(16, a.convs * world))))
        tp = len(topo.replicas[LARGE][0])
        where = "small replicas co-located on the large pool's GPUs" if topology == "colocated" else "disjoint GPU pools"
        model_desc = f"{sm} small x{n_small} + {lg} large TP={tp} ({where})"
        n_convs = a.convs * world
        parallelism = f"{topology}:small{n_small}xtp1+large{len(topo.replicas[LARGE])}xtp{tp}"
        layout = {"small": {"model": sm, "replicas": topo.replicas[SMALL], "tp": 1},
                  "large": {"model": lg, "replicas": topo.replicas[LARGE], "tp": tp},
                  "colocated": topology == "colocated"}

    t_ready = time.perf_counter()   # engines built, weights initialised, GEMMs tuned, graphs captured

    def sync():
        if cluster is not None:
            cluster.sync()
            return
        if on_gpu:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    # this rank's GPU energy over the timed window (amdsmi's cumulative energy counter; no sampling
    # thread): board energy per generated token next to the reference's J/token
    meter, smi_idx, e0 = None, None, None
    busy = None      # sampled GPU busy share over the window (amdsmi activity counter)
    if on_gpu:
        from distributed_llm_amd.bench.power import BusySampler, PowerSampler, smi_index_for_cuda
        smi_idx = smi_index_for_cuda(local)
        meter = PowerSampler(gpus=[smi_idx])
        if not meter.available:
            meter = None
        busy = BusySampler(smi_idx)
    busy_pct = None
    records = []
    tokens = 0
    elapsed = 0.0
    st0 = st1 = None
    e1 = None
    t_window0 = None
    if cluster is not None and rank != 0:
        if meter:
            e0 = meter.mark()
        cluster.serve()  # returns when the router stops the pools
        e1 = meter.mark() if meter else None
        ts = cluster.sync_times
        elapsed = ts[-1] - ts[-2] if len(ts) >= 2 else 0.0
    else:
        pools_for_router = cluster.router_pools() if cluster is not None else pools
        router = Router(strategy=a.strategy, config=cfg, threshold_fallback=a.threshold, benchmark_mode=False,
                        pools=pools_for_router)
        pipelined = bool(a.pipeline)
        if pipelined:
            # the engine's step loop and the routing driver are two Python threads: a short GIL
            # switch interval (0.5 ms; Python's default is 5) hands the GIL back to the step loop
            # before the queued decode step runs dry (+1-1.4 % routed tok/s, profiles/r4_driver_window_gaps.md)
            sys.setswitchinterval(a.gil_switch_ms / 1000.0)
            for e in engines:
                e.ADMIT_EVERY = max(1, a.admit_every)
                e.start()              # background step loop: callers only enqueue and wait
            convs = EventConversations(n_convs, rank) if a.pipeline == 2 else PipelinedConversations(n_convs, rank)
            convs.start(router)
            convs.wait_turns(a.warmup * n_convs)
        else:
            convs = Conversations(n_convs, rank)
            for _ in range(a.warmup):
                convs.step(router)
        if pipelined:
            # steady-state window: the turns completing from here on are the timed ones; the node
            # barrier (cluster: every pool rank records it as its window start) opens it everywhere
            if cluster is not None:
                cluster.sync()
            elif world > 1:
                dist.barrier()         # replicas open their windows together
            with convs._cv:
                st0 = [dict(e.stats()) for e in engines]
                enc0 = encoder_stats()
                if on_gpu:
                    torch.cuda.synchronize()
                e0 = meter.mark() if meter else None
                if busy is not None:
                    busy.start()
                cpu0 = _thread_cpu() if diag("cpu") else None
                t0 = time.perf_counter()
                t_window0 = t0
                convs.records = records
                start_count = convs.completed   # (turns completed during the opening barrier are warmup)
            convs.wait_turns(start_count + a.steps * n_convs)
            with convs._cv:
                convs.records = None
                if on_gpu:
                    torch.cuda.synchronize()
                elapsed = time.perf_counter() - t0
                cpu1 = _thread_cpu() if cpu0 is not None else None
                e1 = meter.mark() if meter else None
                busy_pct = busy.stop() if busy is not None else None
                st1 = [dict(e.stats()) for e in engines]
                enc1 = encoder_stats()
            if cluster is not None:
                cluster.sync()         # closes the pool ranks' windows
            convs.stop()
        else:
            st0 = [dict(e.stats()) for e in engines]
            enc0 = encoder_stats()
            sync()
            e0 = meter.mark() if meter else None
            if busy is not None:
                busy.start()
            t0 = time.perf_counter()
            t_window0 = t0
            dump = [] if a.dump_responses else None
            for _ in range(a.steps):
                convs.step(router, records, dump)
            if dump is not None:
                with open(a.dump_responses, "w") as f:
                    json.dump(dump, f)
            sync()
            elapsed = time.perf_counter() - t0
            e1 = meter.mark() if meter else None
            busy_pct = busy.stop() if busy is not None else None
            st1 = [dict(e.stats()) for e in engines]
            enc1 = encoder_stats()
        if cluster is not None:
            cluster.shutdown()
        for e in engines:
            e.stop()
        tokens = sum(r["tok"] for r in records)
    lats = sorted(r["lat"] for r in records)
    energy_j = -1.0
    if meter and e0 is not None and e1 is not None:
        mj, how = meter.energy_between([smi_idx], e0, e1)
        energy_j = mj / 1000.0 if how == "counter" else -1.0
    if rehearse and rank != 0 and energy_j >= 0:
        energy_j = 0.0   # every rank read the SAME card's counter: count it once (rank 0's)
    dead_ranks = []
    degraded = bool(cluster is not None and cluster.degraded)
    # replicated ranks also reduce (tokens, window) through the process group's own collectives
    # (RCCL on a GPU node: the driver's N > 1 runs then execute RCCL all-reduces across devices)
    # and rank 0 checks them against the store reduction below
    coll = _collective_cross_check(tokens, elapsed, dev, world) if (
        world > 1 and not rehearse and topology == "replicated" and not degraded) else None
    if world > 1:
        # cross-rank reduction through the rendezvous store (hosted by rank 0's process): a pool
        # rank lost mid-run (fault injection, a dead GPU) leaves a missing key instead of hanging
        # a collective; rank 0 reduces whatever the survivors reported
        import datetime
        store = dist.distributed_c10d._get_default_store()
        store.set(f"dllm_bench/{rank}", json.dumps({"tokens": float(tokens), "elapsed": elapsed, "energy": energy_j,
                                                    "lats": lats, "init_s": t_ready - _T_PROC0,
                                                    "startup_s": (t_window0 or t_ready) - _T_PROC0,
                                                    "mem_gb": _peak_mem_gb(on_gpu)}))
        tokens_all, elapsed_max, e_sum, e_bad = 0.0, 0.0, 0.0, False
        init_max, startup_max = t_ready - _T_PROC0, (t_window0 or t_ready) - _T_PROC0
        if rank == 0:
            got = []
            for r in range(world):
                try:
                    store.wait([f"dllm_bench/{r}"], datetime.timedelta(seconds=60 if not degraded else 10))
                    got.append(json.loads(store.get(f"dllm_bench/{r}")))
                except Exception:  # noqa: BLE001 - this rank never reported: it died
                    dead_ranks.append(r)
            tokens_all = sum(g["tokens"] for g in got)
            elapsed_max = max(g["elapsed"] for g in got)
            e_bad = any(g["energy"] < 0 for g in got) or bool(dead_ranks)
            energy_j = -1.0 if e_bad else sum(g["energy"] for g in got)
            lats = sorted(x for g in got for x in g["lats"])
            init_max = max([init_max] + [g.get("init_s", 0.0) for g in got])
            startup_max = max([startup_max] + [g.get("startup_s", 0.0) for g in got])
            rank_mem_gb = [g.get("mem_gb") for g in got]
            degraded = degraded or bool(dead_ranks)
    else:
        tokens_all, elapsed_max = float(tokens), elapsed
        init_max, startup_max = t_ready - _T_PROC0, (t_window0 or t_ready) - _T_PROC0
        rank_mem_gb = [_peak_mem_gb(on_gpu)]
    if rank == 0:
        value = tokens_all / max(elapsed_max, 1e-9)
        rates = sorted(r["tok"] * 1000.0 / r["lat"] for r in records if r["lat"] > 0 and r["tok"] > 0)
        per_stream = rates[len(rates) // 2] if rates else None   # one request's own decode rate (reference protocol)
        pct = lambda p: lats[min(len(lats) - 1, int(p * len(lats)))] if lats else 0.0
        n_small = sum(1 for r in records if r["dev"] == SMALL)
        hits = sum(b["prefix_hit_tokens"] - a_["prefix_hit_tokens"] for a_, b in zip(st0, st1))
        prompt = sum(b["prompt_tokens"] - a_["prompt_tokens"] for a_, b in zip(st0, st1))
        out = {
            "metric": "routed_tokens_per_sec",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed_max * 1000.0 / a.steps, 2),
            "higher_is_better": True,
            "scaling": "weak" if topology in ("replicated", "tiers") else "config",
            "vs_baseline": round(value / BASELINE_TOK_S, 2),
            # vs_baseline divides this whole-job aggregate (all conversations, all GPUs) by the
            # reference's single-stream 10.57 tok/s; the like-for-like ratio is per stream:
            "vs_baseline_basis": "aggregate tokens/s over all concurrent conversations / reference single-stream "
                                 "10.57 tok/s (BASELINE.md)",
            "per_stream_tok_s_p50": round(per_stream, 1) if per_stream else None,
            "per_stream_vs_baseline": round(per_stream / BASELINE_TOK_S, 2) if per_stream else None,
            "baseline_config": baseline_config,
            "layout": layout,
            "per_gpu_tok_s": round(value / max(1, world), 2),
            # process start -> engines ready (weights init, GEMM autotune, graph capture); -> timed window
            # (plus the warmup turns); max over ranks
            "collective_cross_check": (dict(coll, matches_store=bool(
                "tokens_sum" in coll and abs(coll["tokens_sum"] - tokens_all) < 0.5
                and abs(coll["elapsed_max_s"] - elapsed_max) < 1e-6)) if coll else None),
            "init_s": round(init_max, 1),
            "peak_device_mem_gb_by_rank": rank_mem_gb,
            "startup_s": round(startup_max, 1),
            "scaling_note": ("every N runs BASELINE config 2 by default (one engine + routing driver per GPU, "
                             "--convs conversations each): per-GPU work is fixed, so values at N = 1..8 are one "
                             "workload's weak-scaling curve; BASELINE's multi-GPU configs run with "
                             "--baseline-config 3 (2 GPUs), 4 (4-8 GPUs), 5 (co-located Mixtral TP=N) and are "
                             "different models and layouts, not points of that curve"
                             if topology == "replicated" else
                             "BASELINE config %d (%s): a different model pair and layout than config 2, not a "
                             "point of the config-2 weak-scaling curve (the default at every N)"
                             % (baseline_config, topology)),
            "dtype": "bf16",
            "data": "synthetic: reference query sets replayed as growing conversations; random-init weights",
            "config": {"model": model_desc, "global_batch": a.convs * world,
                       "seq_len": "growing conversation (<=16384)", "parallelism": parallelism,
                       "decode_graphs": bool(engines) and all(getattr(e, "use_graphs", False) for e in engines),
                       # (rank 0's engines; in a one-GPU rehearsal only TP tiers run eager)
                       "strategy": a.strategy, "semantic_cache": True, "response_cache": False,
                       "perf_explore": bool(cfg.get("perf_explore")),
                       "penalise_failed_primary": bool(cfg.get("penalise_failed_primary")),
                       "turn_pipelining": (("event-driver" if a.pipeline == 2 else "thread-per-conversation")
                                           if a.pipeline else False),
                       "admit_every": a.admit_every if a.pipeline else None,
                       "gil_switch_ms": a.gil_switch_ms if a.pipeline else None,
                       "small_max_new": a.small_new, "large_max_new": a.large_new},
            # client side, as the reference harness times a turn (routing_chatbot_tester.py:408-442):
            # dispatch (routing included) to the answer being back in the driver, failover included
            "p50_latency_ms": round(statistics.median(lats), 1) if lats else None,
            "latency_basis": "client: turn dispatched -> answer collected (routing, queueing, failover included)",
            "p50_engine_latency_ms": (round(statistics.median(r["lat_engine"] for r in records), 1)
                                      if records and all("lat_engine" in r for r in records) else None),
            "p90_latency_ms": round(pct(0.9), 1),
            "p50_speedup_vs_baseline_mean_latency": (round(BASELINE_S_PER_QUERY * 1000.0 / statistics.median(lats), 1)
                                                     if lats else None),
            "requests": len(lats),
            "small_tier_share": round(n_small / max(1, len(records)), 3),
            "routing_overhead_ms_mean": round(statistics.mean(r["ovh"] for r in records), 3) if records else None,
            "ttft_ms_p50": round(statistics.median(r["ttft"] for r in records), 1) if records else None,
            "prefix_cache_hit_rate": round(hits / max(1, prompt), 3),
            # new KV blocks that continued their sequence's run / opened a free segment / other
            # (csrc/runtime/block_manager.h fresh(); profiles/r5_kv_placement.md)
            "kv_block_placement": kv_placement(st0, st1),
            "engine_decode_tok_s": round(sum(b["decode_tokens"] - a_["decode_tokens"] for a_, b in zip(st0, st1))
                                         / max(elapsed_max, 1e-9), 1),
            "avg_decode_batch": round(sum(b["decode_tokens"] - a_["decode_tokens"] for a_, b in zip(st0, st1))
                                      / max(1, sum(b["decode"] - a_["decode"] for a_, b in zip(st0, st1))), 1),
            "engine_time_split_s": engine_time_split(st0, st1, elapsed_max),
        }
        if busy_pct is not None:
            # rank 0's GPU, sampled at 20 Hz over the timed window (no kernel trace: a traced run's
            # host is slower and shows idle gaps the plain run does not have)
            out["gpu_busy_sampled_pct"] = round(busy_pct, 1)
        if energy_j >= 0:
            # every rank's GPU over the timed window (energy counter deltas summed over ranks)
            out["gpu_energy_j"] = round(energy_j, 1)
            out["avg_gpu_power_w"] = round(energy_j / max(elapsed_max, 1e-9) / (1 if rehearse else world), 1)
            out["j_per_token"] = round(energy_j / max(tokens_all, 1.0), 4)
        if rehearse:
            out["rehearsal_one_gpu"] = True   # N ranks shared ONE GPU: plumbing check, not a number
        if a.layers:
            out["truncated_layers"] = a.layers   # not the named models' full depth: not a number either
        fo = [r for r in records if r.get("fo")]
        dead_tiers = sorted({r["fo"] for r in fo})
        first_fo = min((r["step"] for r in fo), default=None)
        out["pool_events"] = {
            "failovers": len(fo), "lost_turns": sum(1 for r in records if not r.get("ok", True)),
            "dead_ranks": dead_ranks, "degraded": degraded, "failed_tiers": dead_tiers,
            "first_failover_step": first_fo,
            # failed-over turns per step from the first failover on (a tier known to be down is
            # skipped up front: those turns still count here, they are served by the other tier)
            "failovers_by_step": (
                [sum(1 for r in fo if r["step"] == st) for st in range(first_fo, max(r["step"] for r in fo) + 1)]
                if first_fo is not None else [])}
        lk = enc1["lookups"] - enc0["lookups"]
        out["router_encoder"] = {"kinds": enc1["kinds"], "memo": bool(enc1.get("memo_enabled", False)),
                                 "lookups": lk, "memo_hit_rate": round((enc1["hits"] - enc0["hits"]) / lk, 3) if lk else None,
                                 "texts_encoded_in_window": enc1["encoded_texts"] - enc0["encoded_texts"],
                                 "batch_reuse_hits": enc1["batch_hits"] - enc0["batch_hits"]}
        if pipelined and cpu1 is not None:   # share of the window each thread spent on a core
            out["thread_cpu_share"] = {k: round((v - cpu0.get(k, 0.0)) / elapsed, 3) for k, v in cpu1.items()
                                       if v - cpu0.get(k, 0.0) > 0.01 * elapsed}
        logs = [e._sync_log for e in engines if getattr(e, "_sync_log", None)]
        if logs:   # DLLM_DIAG=sync diagnostics: did the step loop keep a step queued ahead?
            import numpy as np
            rec = np.array([r for lg in logs for r in lg], dtype=np.float64)
            wait = rec[:, 1] * 1e3
            out["step_loop_sync"] = {"steps": int(len(rec)), "prep_ms_p50": round(float(np.median(rec[:, 0]) * 1e3), 3),
                                     "wait_ms_p50": round(float(np.median(wait)), 3),
                                     "wait_under_0.1ms": int((wait < 0.1).sum()),
                                     "wait_ms_pcts": [round(float(x), 3) for x in np.percentile(wait, [5, 25, 75, 95])]}
        print(json.dumps(out), flush=True)
    if a.trace:
        from distributed_llm_amd.utils.tracing import tracer
        tracer.dump()
    if world > 1:
        if degraded:
            # a peer is gone: no further collectives (they would fail or hang); leave without the
            # process-group teardown handshake
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0)
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
