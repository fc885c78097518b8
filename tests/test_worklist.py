"""Decode attention work list (ops.decode_work_items): every (tile, kv head) key range is covered
by exactly its ``nsplit`` units, split counts are bounded, and the list size tracks the target."""
import numpy as np
import pytest

from distributed_llm_amd import ops


@pytest.mark.parametrize("nkv,max_splits,target,min_chunk", [(4, 16, 2048, 256), (8, 16, 64, 32), (1, 4, 10_000, 32)])
def test_work_items_cover_every_tile(nkv, max_splits, target, min_chunk):
    rng = np.random.default_rng(0)
    ctx = np.sort(rng.integers(1, 9000, size=300))[::-1]
    buf = ops.decode_work_items(ctx, nkv, max_splits, target, min_chunk=min_chunk)
    n = int(buf[0])
    w = buf[1:1 + 2 * n].reshape(n, 2).astype(np.int64)
    tile, kvh = w[:, 0] & 0xFFFF, w[:, 0] >> 16
    split, ns = w[:, 1] & 0xFF, w[:, 1] >> 8
    assert (ns >= 1).all() and (ns <= max_splits).all() and (split < ns).all() and (kvh < nkv).all()
    seen = {}
    for t, h, s_, n_ in zip(tile, kvh, split, ns):
        seen.setdefault((t, h), set()).add((s_, n_))
    assert len(seen) == len(ctx) * nkv
    for (t, h), units in seen.items():
        n_ = {u[1] for u in units}
        assert len(n_) == 1
        assert {u[0] for u in units} == set(range(n_.pop()))
    # units are emitted tile by tile (longest tile first when ctx is sorted descending)
    assert (np.diff(tile) >= 0).all()
    chunk = max(min_chunk, -(-int(ctx.sum()) * nkv // target))
    if ctx.max() / chunk < max_splits:
        assert n <= ctx.size * nkv + int(ctx.sum()) * nkv // chunk + 1


def test_work_items_into_buffer():
    out = np.full(1 + 2 * 64, -7, dtype=np.int32)
    buf = ops.decode_work_items(np.array([100, 40]), 2, 16, 64, min_chunk=32, out=out)
    assert buf is out and int(out[0]) == 2 * (4 + 2)   # ceil(100/32)=4, ceil(40/32)=2 splits


def test_work_items_extended_form():
    """Extended list: -n, 3 pad words, then 16-B units that also carry (seq | qstart << 16, ctx)
    of their tile; the (tile, head, split) part is identical to the plain list."""
    ctx = np.array([900, 300, 40, 1])
    seq = np.array([5, 0, 7, 2])
    qstart = np.array([1, 3, 0, 2])
    plain = ops.decode_work_items(ctx, 4, 16, 64, min_chunk=64)
    ext = ops.decode_work_items(ctx, 4, 16, 64, min_chunk=64, seq=seq, qstart=qstart)
    n = int(plain[0])
    assert int(ext[0]) == -n and (ext[1:4] == 0).all() and ops.work_items_len(ext) == 4 + 4 * n == ext.size
    assert ops.work_items_len(plain) == 1 + 2 * n
    u = ext[4:].reshape(n, 4).astype(np.int64)
    assert (u[:, :2] == plain[1:].reshape(n, 2)).all()
    tile = u[:, 0] & 0xFFFF
    assert (u[:, 2] & 0xFFFF == seq[tile]).all() and (u[:, 2] >> 16 == qstart[tile]).all()
    assert (u[:, 3] == ctx[tile]).all()
