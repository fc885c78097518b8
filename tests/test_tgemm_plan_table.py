"""The pruned tgemm plans (csrc/kernels/tgemm.hip kPruned, not instantiated) and the Python mirror
(ops.gemm._TG_PRUNED) are the same table, and nothing the autotuner, the heuristic or the MoE
path asks for is pruned (a pruned plan is refused at launch; profiles/r6_prune.md)."""
import os
import re

import pytest

from distributed_llm_amd import ops
from distributed_llm_amd.ops import gemm as G

SRC = os.path.join(os.path.dirname(__file__), "..", "csrc", "kernels", "tgemm.hip")


def _cpp_table():
    text = open(SRC).read()
    body = text[text.index("constexpr PlanKey kPruned[] = {"):]
    body = body[:body.index("};")]
    return {tuple(int(v) for v in m.split(",")) for m in re.findall(r"\{([\d,\s]+)\}", body)}


def test_cpp_and_python_tables_match():
    cpp = _cpp_table()
    assert cpp and all(len(k) == 9 for k in cpp)
    assert cpp == set(G._TG_PRUNED)


@pytest.mark.parametrize("M", [1, 16, 64, 65, 128, 129, 256, 320, 480, 512, 1024])
@pytest.mark.parametrize("N,K", [(2560, 2048), (2048, 2048), (11264, 2048), (2048, 5632), (6144, 4096),
                                 (4096, 4096), (28672, 4096), (4096, 14336), (32000, 2048)])
def test_candidates_and_heuristic_are_built(M, N, K):
    for c in G._tg_cands(M, N, K):
        assert G.tg_built(c), c
    assert G.tg_built(G.tg_plan(M, N, K))


def test_fixed_plan_lists_are_built():
    for p in G._PF_PLANS + G._TG_M32:
        assert G.tg_built(p), p
    for bm, bn, st, nl in G._TG_K32:
        assert G.tg_built((bm, bn, st, 1, 1, 8, 1, nl, 0, 32))
    for bm, bn, nw, st, nl, _ in G._TG_NL:
        assert G.tg_built((bm, bn, st, 1, 1, nw, 1, nl))
    for p in ops.MOE_PLANS.values():   # (bm, bn13, st13, ks13, nw13, bn2, st2, ks2, nw2)
        assert G.tg_built((p[0], p[1], p[2], 1, p[3], p[4]))
        assert G.tg_built((p[0], p[5], p[6], 1, p[7], p[8]))


def test_gemv_grid_policy_host():
    """Batch 2-8 GEMV grid (csrc/kernels/gemv.hip gemv_grid): capped at max(512, N / 4M) workgroups
    from N = 8192 on, one workgroup per 4R columns otherwise and at batch 1.  Host-side launch
    geometry: the native library answers without a GPU."""
    try:
        ext = ops._load()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"native library not built here: {e}")
    blocks = lambda N, R: -(-N // (4 * R))
    for M in (1, 2, 4, 8):
        for N in (2048, 2560, 6144, 8192, 11264, 28672, 32000, 128256):
            for R in (1, 2, 4):
                want = blocks(N, R) if (M == 1 or N < 8192) else min(blocks(N, R), max(512, -(-N // (4 * M))))
                assert ext.gemv_slots(M, N, R) == want, (M, N, R)
    ext.gemv_set_grid(1, 0, 0)   # policy off: one workgroup per column block everywhere
    try:
        assert ext.gemv_slots(8, 28672, 1) == blocks(28672, 1)
    finally:
        ext.gemv_set_grid(512, 4, 8192)
