"""Host-side rules of the decode path, on CPU: fused-GEMV choice coupling
(ops.gemm._couple_gemv_choices: a residual producer (Wo, down) keeps the fused GEMV only where its
consumer (gate|up, next layer's QKV) runs it too, since a GEMV producer leaves one row-sum slot per
workgroup), fused-GEMV eligibility, and the embedding gather's row sums (reference path)."""
from distributed_llm_amd.ops import gemm as G

LAYER = [(2560, 2048), (2048, 2048), (11264, 2048), (2048, 5632)]   # QKV, Wo, gate|up, down


def _set(M, choices):
    for (N, K), c in zip(LAYER, choices):
        G._P.fused_core[(M, N, K)] = c
        G._P.fused_opts[(M, N, K)] = {"tg": 5.0, "lin": 4.0, c: 3.0}


def test_producer_drops_gemv_when_consumer_does_not_run_it(monkeypatch):
    monkeypatch.setattr(G._P, "fused_core", {})
    monkeypatch.setattr(G._P, "fused_opts", {})
    _set(1, ("gemv1",) * 4)                          # all GEMV: nothing changes
    _set(4, ("gemv1", "gemv1", "tg", "gemv1"))       # Wo -> tg gate|up: Wo falls back, down keeps it
    _set(8, ("lin", "gemv2", "gemv1", "gemv1"))      # down -> lin QKV: down falls back
    G._couple_gemv_choices(LAYER, [1, 4, 8], verbose=False)
    fc = G._P.fused_core
    assert all(fc[(1, N, K)] == "gemv1" for N, K in LAYER)
    assert fc[(4, 2048, 2048)] == "lin" and fc[(4, 2048, 5632)] == "gemv1" and fc[(4, 2560, 2048)] == "gemv1"
    assert fc[(8, 2048, 2048)] == "gemv2" and fc[(8, 2048, 5632)] == "lin"


def test_moe_layers_have_no_pairs(monkeypatch):
    monkeypatch.setattr(G._P, "fused_core", {(2, 2560, 2048): "gemv1", (2, 2048, 2048): "gemv1"})
    monkeypatch.setattr(G._P, "fused_opts", {})
    G._couple_gemv_choices(LAYER[:2], [2], verbose=False)
    assert G._P.fused_core[(2, 2048, 2048)] == "gemv1"


def test_fused_gemv_eligibility(monkeypatch):
    """fused_gemv_r: only batch 1/2/4/8, X within the 64 KB LDS stage, 16-B aligned rows, N % 32 == 0,
    and only where the autotuner (or DLLM_FUSED_CORE) picked a gemvR core."""
    import torch
    monkeypatch.setattr(G._P, "fused_core", {(1, 2560, 2048): "gemv2", (8, 2560, 2048): "tg"})
    monkeypatch.delenv("DLLM_FUSED_CORE", raising=False)
    x1 = torch.zeros(1, 2048, dtype=torch.bfloat16)
    assert G.fused_gemv_r(x1, 2560) == 2
    assert G.fused_gemv_r(torch.zeros(8, 2048, dtype=torch.bfloat16), 2560) == 0     # tuned to tgemm
    assert G.fused_gemv_r(torch.zeros(3, 2048, dtype=torch.bfloat16), 2560) == 0     # not a GEMV batch
    assert G.fused_gemv_r(x1, 2561) == 0                                             # N % 32
    assert G.fused_gemv_r(torch.zeros(8, 8192, dtype=torch.bfloat16), 2560) == 0     # 128 KB of X
    assert G.fused_gemv_r(torch.zeros(1, 4096, dtype=torch.bfloat16)[:, :2048], 2560) == 2   # strided rows ok
    monkeypatch.setenv("DLLM_FUSED_CORE", "gemv4")
    assert G.fused_gemv_r(torch.zeros(4, 2048, dtype=torch.bfloat16), 64) == 4
    monkeypatch.setenv("DLLM_FUSED_CORE", "tg")
    assert G.fused_gemv_r(x1, 2560) == 0


def test_embedding_row_sums_reference_path():
    """ops.embedding(ssq_out=...) on CPU: the gathered rows and each row's sum of squares (the
    first decoder layer's row scale input), zero rows for ids outside the vocab shard."""
    import torch
    from distributed_llm_amd import ops
    table = torch.randn(50, 64).to(torch.bfloat16)
    ids = torch.tensor([3, 7, 49, 60, 0], dtype=torch.int32)
    ssq = torch.full((8,), float("nan"))
    out = ops.embedding(ids, table, 0, ssq_out=ssq)
    want = torch.stack([table[i] if i < 50 else torch.zeros(64, dtype=torch.bfloat16) for i in ids.tolist()])
    assert torch.equal(out, want)
    torch.testing.assert_close(ssq[:5], (want.float() ** 2).sum(1))
    assert torch.isnan(ssq[5:]).all()
