"""Host-side op dispatch rules (no GPU needed)."""
from distributed_llm_amd import ops


def test_flash_supported_applies_the_launchers_lds_bound():
    # the flash kernel stages a tile's whole block-table row next to its K/V ring in the 160 KB
    # LDS: tables that do not fit must fall back to the paged kernel instead of failing at launch
    for d in (64, 96, 128):
        assert ops.flash_supported(d, 4, 1024)
        fit = max(b for b in range(1, 60000, 64) if ops.flash_lds_bytes(d, b) <= 160 * 1024)
        assert ops.flash_supported(d, 4, fit) and not ops.flash_supported(d, 4, fit + 64)
    assert ops.flash_lds_bytes(128, 8192) == 3 * 2 * 64 * 128 * 2 + 8192 * 4
    assert not ops.flash_supported(80, 4, 16) and not ops.flash_supported(128, 3, 16)


def test_flash_split_heuristic(monkeypatch):
    """Flash split-KV is chosen only for a small grid over a long context (measured slower on cold
    short prompts, 1.5-5x faster on a turn's new tokens over a long cached history:
    profiles/r4_flash_split.md); DLLM_FLASH_SPLITS forces a factor (1 = off, capped at 16)."""
    monkeypatch.delenv("DLLM_FLASH_SPLITS", raising=False)
    assert ops.flash_splits(20, 2048) == 1          # short context: never
    assert ops.flash_splits(300, 32768) == 1        # the grid already fills the chip
    assert ops.flash_splits(20, 4096) == 2 and ops.flash_splits(20, 16384) == 8
    assert ops.flash_splits(128, 16384) == 4        # capped by the 512-workgroup target
    monkeypatch.setenv("DLLM_FLASH_SPLITS", "3")
    assert ops.flash_splits(1000, 0) == 3
    monkeypatch.setenv("DLLM_FLASH_SPLITS", "99")
    assert ops.flash_splits(1, 0) == 16


def test_sample_split_policy():
    """Split-vocab sampler only for small batches of large-vocab rows (profiles/r4_sampler.md)."""
    from distributed_llm_amd import ops
    assert ops.sample_split_shards(1, 32000) == 1          # TinyLlama: one workgroup per row
    assert ops.sample_split_shards(1, 128256) == 8         # Llama-3: 8 shards of ~16K
    assert ops.sample_split_shards(ops.SAMPLE_SPLIT_MAX_B + 1, 128256) == 1
    assert ops.sample_split_shards(4, 65536) == 8 and ops.sample_split_shards(4, 65535) == 1
