"""Engine scheduling on CPU (tiny random model, torch reference ops): continuous batching across
concurrent callers, and the pool-side Coalescer."""
import threading
import time

import pytest

from distributed_llm_amd.engine.llm_engine import LLMEngine
from distributed_llm_amd.engine.sampling import SamplingParams
from distributed_llm_amd.pools.base import Coalescer


@pytest.fixture(scope="module")
def engine():
    return LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=16, seed=0)


def test_concurrent_callers_share_one_batch(engine):
    n, new = 6, 12
    prompts = [f"user: question number {i} about topic {i * 7}\nassistant: " for i in range(n)]
    sp = SamplingParams(max_new_tokens=new, temperature=0.0, ignore_eos=True)
    results = [None] * n
    start = threading.Barrier(n)

    def call(i):
        start.wait()
        results[i] = engine.generate([prompts[i]], sp)[0]

    before = dict(engine.steps)
    ts = [threading.Thread(target=call, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert all(r is not None and r.error is None for r in results)
    assert all(r.num_generated == new for r in results)
    decode_steps = engine.steps["decode"] - before["decode"]
    # serial execution would need n * (new - 1) decode steps; merged callers share steps
    assert decode_steps < n * (new - 1)
    assert not engine._driving and not engine._inbox


def test_concurrent_results_match_single_batch(engine):
    sp = SamplingParams(max_new_tokens=8, temperature=0.0, ignore_eos=True)
    prompts = ["user: alpha beta gamma\nassistant: ", "user: delta epsilon\nassistant: "]
    ref = [o.token_ids for o in engine.generate(prompts, sp)]
    out = [None, None]

    def call(i):
        out[i] = engine.generate([prompts[i]], sp)[0].token_ids

    ts = [threading.Thread(target=call, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert out == ref


def test_coalescer_merges_waiting_callers():
    sizes = []

    def fn(items):
        sizes.append(len(items))
        time.sleep(0.2 if len(sizes) == 1 else 0.0)
        return [x * 2 for x in items]

    c = Coalescer(fn)
    out = {}
    first = threading.Thread(target=lambda: out.__setitem__(-1, c.submit([100])))
    first.start()
    time.sleep(0.05)  # the first call is now in flight
    ts = [threading.Thread(target=lambda i=i: out.__setitem__(i, c.submit([i, i + 1000]))) for i in range(7)]
    for t in ts:
        t.start()
    for t in ts + [first]:
        t.join(timeout=10)
    assert out[-1] == [200]
    for i in range(7):
        assert out[i] == [2 * i, 2 * (i + 1000)]
    assert sum(sizes) == 15 and len(sizes) == 2 and sizes[1] == 14


def test_coalescer_propagates_errors():
    def fn(items):
        raise ValueError("boom")

    with pytest.raises(ValueError):
        Coalescer(fn).submit([1])


def test_background_loop_serves_staggered_callers():
    """Server mode (LLMEngine.start): a caller returns as soon as ITS request is done, while a
    longer request keeps decoding; results equal the leader-driven engine's."""
    eng = LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=16, seed=0)
    short = SamplingParams(max_new_tokens=4, temperature=0.0, ignore_eos=True)
    long_ = SamplingParams(max_new_tokens=40, temperature=0.0, ignore_eos=True)
    p_short, p_long = "user: short one\nassistant: ", "user: a long answer please\nassistant: "
    ref_short = eng.generate([p_short], short)[0].token_ids
    ref_long = eng.generate([p_long], long_)[0].token_ids
    eng.start()
    try:
        out, done_at = {}, {}

        def call(name, p, sp):
            out[name] = eng.generate([p], sp)[0]
            done_at[name] = time.perf_counter()

        tl = threading.Thread(target=call, args=("long", p_long, long_))
        tl.start()
        time.sleep(0.05)
        ts = threading.Thread(target=call, args=("short", p_short, short))
        ts.start()
        ts.join(timeout=120)
        tl.join(timeout=120)
        assert out["short"].token_ids == ref_short and out["long"].token_ids == ref_long
        assert done_at["short"] < done_at["long"]     # the short caller was not held by the long one
        assert eng._driving and eng._bg is not None
    finally:
        eng.stop()
    assert not eng._driving and eng._bg is None
    assert eng.generate([p_short], short)[0].token_ids == ref_short   # leader mode again


def test_submit_notifies_each_finished_request_once():
    """``submit(..., notify=)``: every request reaches the completion queue exactly once, already
    done, with the same tokens as a blocking ``generate`` (the event driver's no-polling path)."""
    import queue
    eng = LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=16, seed=0)
    sps = [SamplingParams(max_new_tokens=n, temperature=0.0, ignore_eos=True) for n in (3, 9, 5, 1)]
    prompts = [f"user: request {i}\nassistant: " for i in range(len(sps))]
    ref = [eng.generate([p], sp)[0].token_ids for p, sp in zip(prompts, sps)]
    eng.start()
    try:
        q = queue.SimpleQueue()
        hs = eng.submit(prompts, sps, notify=q.put)
        got = [q.get(timeout=120) for _ in hs]
        assert sorted(map(id, got)) == sorted(map(id, hs)) and q.empty()
        assert all(h.done.is_set() for h in got)
        assert [o.token_ids for o in eng.results(hs)] == ref
    finally:
        eng.stop()


def test_seq_finish_notifies_once():
    """a row that stops inside a pipelined burst is finished by ``_complete_early`` and
    again by ``_release``; the completion callback must still fire exactly once."""
    from distributed_llm_amd.engine.llm_engine import _Seq
    calls = []
    s = _Seq(id=7, prompt=[1, 2], params=SamplingParams(), arrival=0.0, notify=calls.append)
    s.finish()
    s.finish()
    assert calls == [s] and s.done.is_set()
    eng = LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=4, seed=0)
    calls.clear()
    sp = SamplingParams(max_new_tokens=4, temperature=0.0, ignore_eos=True)
    eng.start()
    try:
        hs = eng.submit(["user: x\nassistant: "], [sp], notify=calls.append)
        for h in hs:
            assert h.done.wait(60)
    finally:
        eng.stop()
    for h in hs:
        eng._complete_early(h)   # a second completion path on an already-finished sequence
    assert calls == hs


def test_route_concurrent_matches_route_query():
    from distributed_llm_amd.config import BENCHMARK_CFG, LARGE, SMALL
    from distributed_llm_amd.orchestrator import Router
    from distributed_llm_amd.pools.base import EchoPool
    pools = {SMALL: EchoPool(SMALL), LARGE: EchoPool(LARGE, tokens_per_reply=48)}
    a = Router("heuristic", config=dict(BENCHMARK_CFG), pools=pools)
    b = Router("heuristic", config=dict(BENCHMARK_CFG), pools=pools)
    hs = [[{"role": "user", "content": q}] for q in ("Thank you!", "Write a Python function for knapsack",
                                                      "what is 2+2", "Compare TCP versus UDP")]
    ref = [a.route_query(h) for h in hs]
    got = [None] * len(hs)

    def call(i):
        got[i] = b.route_concurrent(hs[i])

    th = [threading.Thread(target=call, args=(i,)) for i in range(len(hs))]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    for (p1, t1, d1), (p2, t2, d2) in zip(ref, got):
        assert (p1["response"], t1, d1, p1["routing_method"]) == (p2["response"], t2, d2, p2["routing_method"])


def test_preemption_under_kv_pressure_completes_every_request():
    """16 KV blocks (256 tokens) for 6 requests needing ~6 blocks each: running sequences run out of
    blocks, are preempted (recompute) and re-admitted; every request still finishes in full."""
    eng = LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.0, max_num_seqs=8, max_model_len=128, seed=0)
    assert eng.num_blocks == 16
    preempts = []
    orig = eng._release

    def counting_release(s, keep=True):
        if not keep:
            preempts.append(s.id)
        return orig(s, keep)

    eng._release = counting_release
    sp = SamplingParams(max_new_tokens=60, temperature=0.0, ignore_eos=True)
    prompts = [f"user: request {i} " + "tok " * (20 + 3 * i) for i in range(6)]
    outs = eng.generate(prompts, sp)
    assert all(o.error is None and o.num_generated == 60 for o in outs), [(o.error, o.num_generated) for o in outs]
    assert preempts, "expected at least one preemption"
    assert eng.bm.check_invariants() == ""
    assert eng.bm.stats()["active_seqs"] == 0


def test_block_table_sync_covers_decode_grown_columns():
    """A row whose block table grew during decode (updates applied inside the step)
    must be fully re-synced when it is released and re-used: the device copy of every row equals
    the host table after the next admission, and the re-used row's output equals a fresh run."""
    eng = LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=1, seed=0)
    sp_long = SamplingParams(max_new_tokens=70, temperature=0.0, ignore_eos=True)
    eng.generate(["user: a\nassistant: "], sp_long)         # grows ~5 blocks during decode
    assert eng._bt_hw >= 5
    sp = SamplingParams(max_new_tokens=40, temperature=0.0, ignore_eos=True)
    prompt = "user: the same row again\nassistant: "
    got = eng.generate([prompt], sp)[0].token_ids
    eng._bt_dirty = True
    eng._sync_bt()
    assert (eng.bt_dev.cpu()[:, :eng._bt_hw] == eng.bt_host_t[:, :eng._bt_hw]).all()
    fresh = LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.05, max_num_seqs=1, seed=0)
    assert got == fresh.generate([prompt], sp)[0].token_ids


def test_block_manager_places_sequences_in_runs():
    """KV blocks of one sequence come out as consecutive runs (each new sequence starts a wholly
    free 64-block segment, growth continues after its last block), also when sequences grow
    interleaved and a later turn re-matches the cached prefix; the LIFO policy stays available."""
    from distributed_llm_amd.engine.llm_engine import _need_runtime
    rt = _need_runtime()
    bm = rt.BlockManager(2000, 16, True)
    ids = list(range(6))
    for i in ids:
        assert bm.allocate(i, list(range(1000 * i + 1, 1000 * i + 40)))[0]
    for _ in range(300):                       # interleaved decode growth
        bm.commit_append(ids, [5] * 6, [1] * 6)
    for i in ids:
        t = bm.block_table(i)
        assert t == list(range(t[0], t[0] + len(t))), t
    st = bm.stats()
    assert st["segment_allocs"] == 6 and st["contiguous_allocs"] > 100
    assert bm.check_invariants() == ""
    # next turn of conversation 0: the history blocks are matched, the new ones continue the run
    hist = list(range(1, 40)) + [5] * 300
    t0 = bm.block_table(0)
    bm.commit(0, len(hist))
    bm.free(0)
    t, cached = bm.allocate(100, hist + list(range(7000, 7100)))
    assert cached > 0 and t[:len(t0) - 1] == t0[:len(t0) - 1]
    assert t == list(range(t[0], t[0] + len(t)))
    assert bm.check_invariants() == ""
    lifo = rt.BlockManager(2000, 16, True, False)
    for i in ids:
        lifo.allocate(i, list(range(1000 * i + 1, 1000 * i + 40)))
    for _ in range(40):
        lifo.commit_append(ids, [5] * 6, [1] * 6)
    assert lifo.stats()["segment_allocs"] == 0 and lifo.check_invariants() == ""


def test_kv_runs_hold_under_eviction_pressure():
    """Round-6 placement (block_manager.h fresh / pop_roomy_segment): on the flagship's KV traffic
    (growing conversations re-sent whole every turn, stale previous-turn decode blocks, a pool the
    cached histories fill, idle gaps between a conversation's turns) most new blocks continue their
    sequence's run, with the same prefix-cache hit rate as plain LIFO placement
    (scripts/kv_placement_sim.py)."""
    import importlib.util
    import pathlib
    spec = importlib.util.spec_from_file_location(
        "kvsim", pathlib.Path(__file__).resolve().parents[1] / "scripts" / "kv_placement_sim.py")
    sim = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sim)
    for gap in ((0, 0), (5, 40)):   # next turn dispatched at once / after a routing + admission gap
        runs = sim.simulate(64, 5000, contiguous=True, gap=gap)   # ~360 blocks per conversation, as the bench
        lifo = sim.simulate(64, 5000, contiguous=False, gap=gap)
        assert runs["invariants"] == "ok" and lifo["invariants"] == "ok"
        assert runs["run_share"] >= 0.75, runs
        assert runs["inplace_share"] > 0.1 and runs["roomy_segment_share"] > 0.0, runs
        # out-of-LRU-order eviction only of cold blocks and of a sequence's own stale continuation:
        # the prefix cache keeps what LRU placement keeps
        assert runs["prefix_hit_rate"] >= lifo["prefix_hit_rate"] - 0.01, (runs, lifo)
