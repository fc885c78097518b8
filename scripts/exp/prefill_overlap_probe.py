"""Does a prefill chunk overlap with decode steps on one MI355X?  (feasibility probe for running the
admission prefill on a side stream while the decode burst continues)

Engine A holds B decode rows at context C and replays its captured decode graph; engine B (its own
weights and KV pool) prefills P sequences of Q new tokens on top of a cached prefix of X tokens --
the flagship's admission chunk (~30 turns x ~130 new tokens behind ~1.7K cached tokens).  Per trial:
  decode   : K decode-step replays alone
  prefill  : one prefill chunk alone (eager, like the engine's prefill step)
  serial   : the two one after the other on one stream
  overlap  : decode replays on stream 1, the prefill on stream 2, one join
overlap well below serial means the MFMA-bound prefill GEMMs fill what the HBM-bound decode
attention and the L2-bound decode GEMMs leave idle.
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts", "exp"))
from distributed_llm_amd import ops  # noqa: E402
from distributed_llm_amd.engine.llm_engine import LLMEngine  # noqa: E402
from distributed_llm_amd.models.llama import AttnMeta  # noqa: E402
from two_graph_overlap import prepare, timed  # noqa: E402

BS = 16


def prefill_fn(eng, P, Q, X, base):
    """Fabricate P prefix-cached sequences (X cached + Q new tokens) in eng and return a closure
    that runs their prefill chunk (hidden states of the new tokens + the LM head of the last ones)."""
    G = eng.model.nq // eng.model.nkv
    flash = ops.flash_supported(eng.model.d, G, eng.max_blocks)
    tiler = ops.flash_tiles if flash else ops.build_tiles
    ids, pos, slots, qstart, qlen, ctx, last, tseq, ttok, rows = [], [], [], [], [], [], [], [], [], []
    t = 0
    for i in range(P):
        sid = base + i
        toks = [5 + (i * 7 + j) % 1000 for j in range(X + Q)]
        tbl, _ = eng.bm.allocate(sid, toks)
        assert tbl, "KV cache too small"
        row = eng._free_rows.pop()
        bt = eng.bm.block_table(sid)
        eng.bt_host[row, :len(bt)] = bt
        rows.append(row)
        ids.extend(toks[X:])
        pos.extend(range(X, X + Q))
        slots.extend(eng.bm.slots(sid, X, X + Q))
        qstart.append(t)
        qlen.append(Q)
        ctx.append(X + Q)
        t += Q
        last.append(t - 1)
        ts, tt = tiler([Q], G)
        tseq.extend([i] * len(ts))
        ttok.extend(tt)
    nb = (X + Q + BS - 1) // BS
    dev = eng.device
    T = lambda x, dt=torch.int32: torch.tensor(np.asarray(x), dtype=dt, device=dev)
    bt_d = T(eng.bt_host[np.array(rows), :nb])
    meta = AttnMeta(slots=T(slots), block_tables=bt_d, qstart=T(qstart), qlen=T(qlen), ctx=T(ctx),
                    tile_seq=T(tseq), tile_tok0=T(ttok), last_idx=T(last, torch.int64),
                    splits=eng._splits_for(len(tseq)), xcd_remap=True, flash=flash)
    ids_d, pos_d = T(ids), T(pos)

    def run():
        with ops.gemm.workspace_owner(eng._ws_owner):
            h = eng.model.hidden_states(ids_d, pos_d, meta, eng.kv_caches)
            return eng.model.logits(h)
    return run, t


def main():
    B = int(os.environ.get("PROBE_B", "496"))
    C = int(os.environ.get("PROBE_C", "1800"))
    P = int(os.environ.get("PROBE_P", "30"))
    Q = int(os.environ.get("PROBE_Q", "130"))
    X = int(os.environ.get("PROBE_X", "1700"))
    K = int(os.environ.get("PROBE_K", "4"))
    kw = dict(device="cuda", kv_cache_gb=float(os.environ.get("PROBE_KV_GB", "40")), max_num_seqs=max(B, P))
    ea = LLMEngine("tinyllama-1.1b", **kw)
    eb = LLMEngine("tinyllama-1.1b", seed=1, **kw)
    g = prepare(ea, B, C, 10_000_000)
    pf, ntok = prefill_fn(eb, P, Q, X, 20_000_000)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def decode():
        for _ in range(K):
            g.replay()

    def serial():
        decode()
        pf()

    def overlap():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            for _ in range(K):
                g.replay()
        with torch.cuda.stream(s2):
            pf()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    res = {"B": B, "C": C, "prefill_seqs": P, "new_tokens": ntok, "cached_prefix": X, "decode_steps": K}
    for name, fn in (("decode_ms", decode), ("prefill_ms", pf), ("serial_ms", serial), ("overlap_ms", overlap),
                     ("decode_ms_2", decode), ("overlap_ms_2", overlap)):
        res[name] = round(timed(fn, 10), 3)
    res["hidden_fraction_of_prefill"] = round((res["serial_ms"] - res["overlap_ms"]) / res["prefill_ms"], 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
