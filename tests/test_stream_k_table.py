"""Host-side stream-K work split (ops.gemm.stream_k_table, consumed by csrc/kernels/tgemm.hip):
every (tile, k-step) is covered exactly once, each workgroup gets an equal contiguous share, and a
tile's contributors carry slab indices 0..c-1 in k order with the same contributor count."""
import numpy as np
import pytest

from distributed_llm_amd.ops.gemm import stream_k_table


@pytest.mark.parametrize("M,N,K,bm,bn,ks,grid", [(320, 2048, 2048, 64, 64, 1, 256), (320, 2560, 2048, 64, 64, 2, 256),
                                                 (37, 200, 384, 64, 64, 1, 256), (448, 2048, 5632, 128, 64, 1, 256),
                                                 (320, 11264, 2048, 64, 128, 1, 80), (130, 320, 1024, 64, 64, 1, 7)])
def test_stream_k_table_covers_every_k_step_once(M, N, K, bm, bn, ks, grid):
    tab, cmax = stream_k_table(M, N, K, bm, bn, ks, grid)
    tiles, nkt = -(-M // bm) * -(-N // bn), K // (64 * ks)
    assert tab.shape[0] == grid and tab.shape[2] == 4 and tab.dtype == np.int32
    seen = np.zeros((tiles, nkt), dtype=np.int32)
    per_tile = {}
    shares = []
    for w in range(grid):
        n = 0
        ended = False
        for t, kb, ke, x in tab[w]:
            if t < 0:
                ended = True
                continue
            assert not ended, "segments after the list end"
            assert 0 <= kb < ke <= nkt
            seen[t, kb:ke] += 1
            per_tile.setdefault(t, []).append((kb, x & 0xFFFF, x >> 16))
            n += ke - kb
        shares.append(n)
    assert (seen == 1).all()
    assert max(shares) - min(shares) <= 1          # equal shares of tiles x k-steps
    assert cmax == max(len(v) for v in per_tile.values())
    for t, lst in per_tile.items():
        lst.sort()
        assert [s for _, s, _ in lst] == list(range(len(lst)))      # slab index = k order
        assert all(c == len(lst) for _, _, c in lst)                 # every contributor knows the count
