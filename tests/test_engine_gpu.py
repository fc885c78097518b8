"""Engine-level GPU checks: HIP path vs torch reference path, hipGraph replay vs eager,
prefix-cache reuse vs cold prefill."""
import copy

import pytest
import torch

from distributed_llm_amd.engine.llm_engine import LLMEngine
from distributed_llm_amd.engine.sampling import SamplingParams
from distributed_llm_amd.models.llama import AttnMeta

pytestmark = pytest.mark.gpu

PROMPTS = ["user: hello there", "user: explain the knapsack problem step by step with code",
           "user: " + "long context " * 40, "x"]


def _engine(**kw):
    kw.setdefault("kv_cache_gb", 0.5)
    kw.setdefault("max_num_seqs", 8)
    return LLMEngine("tiny-llama-test", device="cuda", **kw)


def test_graph_replay_matches_eager():
    g = _engine(use_graphs=True)
    e = _engine(use_graphs=False)
    sp = SamplingParams(max_new_tokens=24)
    a = [o.token_ids for o in g.generate(PROMPTS, sp)]
    b = [o.token_ids for o in e.generate(PROMPTS, sp)]
    assert a == b


def test_prefix_cache_matches_cold():
    warm = _engine(prefix_cache=True)
    cold = _engine(prefix_cache=False)
    sp = SamplingParams(max_new_tokens=12)
    first = warm.generate([PROMPTS[2]], sp)[0]
    turn2 = PROMPTS[2] + "\nassistant: " + first.text + "\nuser: and then?"
    w = warm.generate([turn2], sp)[0]
    c = cold.generate([turn2], sp)[0]
    assert w.num_cached >= 16 and c.num_cached == 0
    assert w.token_ids == c.token_ids


def test_hip_forward_matches_torch_reference():
    eng = _engine(use_graphs=False)
    m = eng.model
    ids = eng.encode(PROMPTS[1])
    T = len(ids)
    slots = eng.bm  # allocate through the engine's block manager
    table, _ = slots.allocate(999, ids)
    sl = slots.slots(999, 0, T)
    dev = torch.device("cuda")
    I = lambda x, dt=torch.int32: torch.tensor(x, dtype=dt, device=dev)
    from distributed_llm_amd import ops
    ts, tt = ops.build_tiles([T], m.nq // m.nkv)
    meta = AttnMeta(I(sl), I([table]), I([0]), I([T]), I([T]), I(ts), I(tt), I([T - 1], torch.int64))
    h_gpu = m.hidden_states(I(ids), I(list(range(T))), meta, eng.kv_caches).float().cpu()
    # same weights on the CPU -> torch reference ops
    mc = copy.copy(m)
    mc.device = torch.device("cpu")
    mc.embed, mc.lm_head, mc.final_norm = m.embed.cpu(), m.lm_head.cpu(), m.final_norm.cpu()
    mc.layers = [{k: v.cpu() for k, v in L.items()} for L in m.reference_layers()]
    mc.fused = False
    mc.cos_sin = m.cos_sin.cpu()
    kv = [(k.cpu().clone(), v.cpu().clone()) for k, v in eng.kv_caches]
    C = lambda t: t.cpu()
    meta_c = AttnMeta(*(C(x) for x in (meta.slots, meta.block_tables, meta.qstart, meta.qlen, meta.ctx,
                                        meta.tile_seq, meta.tile_tok0, meta.last_idx)))
    h_cpu = mc.hidden_states(C(I(ids)), C(I(list(range(T)))), meta_c, kv).float()
    slots.free(999)
    torch.testing.assert_close(h_gpu, h_cpu, atol=6e-2, rtol=5e-2)


def test_tinyllama_generate_and_sampling():
    eng = LLMEngine("tinyllama-1.1b", device="cuda", kv_cache_gb=2.0, max_num_seqs=16, max_model_len=4096)
    outs = eng.generate(PROMPTS, [SamplingParams(max_new_tokens=16), SamplingParams(max_new_tokens=9, temperature=0.8, top_k=40, top_p=0.9),
                                  SamplingParams(max_new_tokens=16), SamplingParams(max_new_tokens=3)])
    assert [o.num_generated for o in outs] == [16, 9, 16, 3]
    assert all(o.error is None for o in outs)
    assert all(0 <= t < 32000 for o in outs for t in o.token_ids)


def _stepwise(monkeypatch):
    monkeypatch.setattr(LLMEngine, "PIPELINE", False)


PROMPTS12 = [f"user: question {i} " + "about things " * (i % 5) for i in range(12)]


def test_pipelined_decode_matches_stepwise(monkeypatch):
    """Pipelined decode (one step of host lookahead, tokens gathered on the device) gives the
    same tokens as the step-by-step loop: mixed max_new_tokens (count limits are predicted),
    more requests than rows (admissions between bursts), greedy and seeded sampling."""
    monkeypatch.setattr(LLMEngine, "BURST_JOIN", False)   # the drained-burst schedule is what matches stepwise
    sps = [SamplingParams(max_new_tokens=3 + 5 * (i % 4), ignore_eos=True, temperature=0.0 if i % 3 else 0.8,
                          top_k=40, top_p=0.9) for i in range(12)]
    a = [o.token_ids for o in _engine(max_num_seqs=4).generate(PROMPTS12, sps)]
    _stepwise(monkeypatch)
    b = [o.token_ids for o in _engine(max_num_seqs=4).generate(PROMPTS12, sps)]
    assert a == b
    assert [len(x) for x in a] == [sp.max_new_tokens for sp in sps]


def test_pipelined_decode_preemption_matches_stepwise(monkeypatch):
    """Out of KV blocks mid-decode: the pipelined loop preempts the same sequences (slot
    reservation fails at the look-ahead commit) and the outputs match the step-by-step loop."""
    monkeypatch.setattr(LLMEngine, "BURST_JOIN", False)   # the drained-burst schedule is what matches stepwise
    sp = SamplingParams(max_new_tokens=40, ignore_eos=True)
    prompts = ["user: " + "word " * 30 + str(i) for i in range(6)]

    def run():   # kv_cache_gb=0 -> the minimum pool (max_model_len / 16 + 8 = 24 blocks)
        e = _engine(kv_cache_gb=0.0, max_num_seqs=6, max_model_len=256)
        return [o.token_ids for o in e.generate(prompts, sp)], e

    a, ea = run()
    _stepwise(monkeypatch)
    b, _ = run()
    assert a == b and all(len(x) == 40 for x in a)
    assert ea.bm.check_invariants() == ""


def test_pipelined_decode_eos_zombie_rows(monkeypatch):
    """A sequence that samples EOS is already in the next launched step: that row is discarded.
    Outputs equal the step-by-step loop up to the first EOS step of the batch, end at EOS, and the
    engine's block accounting is clean afterwards."""
    monkeypatch.setattr(LLMEngine, "BURST_JOIN", False)   # the drained-burst schedule is what matches stepwise
    sp = SamplingParams(max_new_tokens=24, ignore_eos=True)
    probe = [o.token_ids for o in _engine().generate(PROMPTS, sp)]
    # an EOS id that some sequences emit early and others late or never
    cand = {}
    for ids in probe:
        for j, t in enumerate(ids[2:12], start=2):
            cand.setdefault(t, j)
    eos = min(cand, key=lambda t: (abs(cand[t] - 5), t))
    sp2 = SamplingParams(max_new_tokens=24)

    def run():
        e = _engine()
        e.tok.eos_id = eos
        return [o.token_ids for o in e.generate(PROMPTS, sp2)], e

    a, ea = run()
    _stepwise(monkeypatch)
    b, _ = run()
    first = min((x.index(eos) for x in b if eos in x), default=24)
    for x, y in zip(a, b):
        assert x[:first + 1] == y[:first + 1]
        assert eos not in x[:-1] and len(x) <= 24
    assert any(x and x[-1] == eos for x in a)
    assert ea.bm.check_invariants() == "" and ea.bm.stats()["active_seqs"] == 0


def test_pipelined_text_and_turn_memo_match_stepwise(monkeypatch):
    """Answers detokenised inside the pipelined burst (under the next GPU step) give the same text
    as the step-by-step loop, and the memoised prompt+answer ids make turn 2 a prefix-cache hit."""
    monkeypatch.setattr(LLMEngine, "BURST_JOIN", False)   # the drained-burst schedule is what matches stepwise
    sps = [SamplingParams(max_new_tokens=6 + 4 * (i % 3), ignore_eos=True) for i in range(len(PROMPTS))]

    def two_turns():
        e = _engine(max_num_seqs=8)
        first = e.generate(PROMPTS, sps)
        turn2 = [p + first[i].text + "\nuser: go on" for i, p in enumerate(PROMPTS)]
        second = e.generate(turn2, sps)
        return [o.text for o in first], [o.token_ids for o in second], [o.num_cached for o in second]

    ta, ia, ca = two_turns()
    _stepwise(monkeypatch)
    tb, ib, cb = two_turns()
    assert ta == tb and ia == ib and ca == cb
    assert all(c >= 16 for c, p in zip(ca, PROMPTS) if len(p) >= 32)


def test_pipelined_short_request_completes_before_long_one():
    """a row that stops inside a pipelined burst is handed back at once (its caller
    wakes, its latency ends) instead of waiting for the longest row of the batch; its KV blocks
    are released after the burst and the block accounting stays clean."""
    import threading
    import time as _time
    e = _engine(max_num_seqs=8).start()
    try:
        done = {}

        def run(name, prompt, n):
            o = e.generate([prompt], SamplingParams(max_new_tokens=n, ignore_eos=True))[0]
            done[name] = (_time.perf_counter(), o)

        ts = [threading.Thread(target=run, args=("long", PROMPTS[1], 200)),
              threading.Thread(target=run, args=("short", PROMPTS[0], 4))]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        (t_short, o_short), (t_long, o_long) = done["short"], done["long"]
        assert o_short.num_generated == 4 and o_long.num_generated == 200
        assert t_short < t_long
        assert o_short.latency_ms < 0.5 * o_long.latency_ms, (o_short.latency_ms, o_long.latency_ms)
    finally:
        e.stop()
    assert e.bm.check_invariants() == "" and e.bm.stats()["active_seqs"] == 0


def test_burst_join_matches_drained_bursts(monkeypatch):
    """BURST_JOIN: requests admitted and prefilled under a running burst join it without a drain,
    and finished rows are released one step later.  Greedy outputs equal the drained-burst
    schedule's (a row's decode numerics do not depend on the rest of the batch), every request gets
    its token count, joins happened, and the block accounting is clean."""
    sps = [SamplingParams(max_new_tokens=3 + 5 * (i % 4), ignore_eos=True) for i in range(12)]
    monkeypatch.setattr(LLMEngine, "ADMIT_EVERY", 2)
    e = _engine(max_num_seqs=4)
    a = [o.token_ids for o in e.generate(PROMPTS12, sps)]
    assert e.steps.get("burst_joins", 0) > 0
    assert e.bm.check_invariants() == "" and e.bm.stats()["active_seqs"] == 0
    assert [len(x) for x in a] == [sp.max_new_tokens for sp in sps]
    monkeypatch.setattr(LLMEngine, "BURST_JOIN", False)
    b = [o.token_ids for o in _engine(max_num_seqs=4).generate(PROMPTS12, sps)]
    assert a == b


def test_burst_join_background_loop_under_load():
    """Background step loop with requests arriving while bursts run (turn pipelining): every
    request completes with its count, none errors, rows and blocks all come back."""
    import threading
    e = _engine(max_num_seqs=6).start()
    outs = []
    lock = threading.Lock()
    try:
        def client(k):
            for t in range(3):
                o = e.generate([PROMPTS12[(k + t) % 12]], SamplingParams(max_new_tokens=4 + (k + t) % 7,
                                                                        ignore_eos=True))[0]
                with lock:
                    outs.append((4 + (k + t) % 7, o))

        ts = [threading.Thread(target=client, args=(k,)) for k in range(10)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
    finally:
        e.stop()
    assert len(outs) == 30
    assert all(o.error is None and o.num_generated == n for n, o in outs)
    assert e.bm.check_invariants() == "" and e.bm.stats()["active_seqs"] == 0
    assert sorted(e._free_rows) == list(range(e.R))
