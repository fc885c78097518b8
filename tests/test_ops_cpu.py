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
