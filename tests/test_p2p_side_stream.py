"""The data plane's side HIP stream (parallel.p2p.side_stream / on_side): RCCL pair-group transfers
run off the compute stream and are complete when the call returns (the reference's probes and
failover hand-offs never wait behind generation: src/router.py:277-282,
src/models/server_manager.py:123-131)."""
import pytest
import torch

from distributed_llm_amd.parallel import p2p


def test_side_stream_is_a_noop_on_cpu():
    assert p2p.side_stream(torch.device("cpu")) is None
    with p2p.on_side(torch.device("cpu")):
        x = torch.arange(4)
    assert x.sum().item() == 6


@pytest.mark.gpu
def test_side_stream_runs_off_the_compute_stream_and_drains_on_exit():
    dev = torch.device("cuda", 0)
    s = p2p.side_stream(dev)
    assert s is p2p.side_stream(torch.device("cuda"))   # one per device
    assert s != torch.cuda.current_stream(dev)
    with p2p.on_side(dev):
        assert torch.cuda.current_stream(dev) == s
        big = torch.empty(64 << 20, dtype=torch.uint8, device=dev).fill_(3)
        total = big[: 1 << 20].sum()
    assert s.query()                                      # drained before on_side returned
    assert torch.cuda.current_stream(dev) != s
    assert int(total.item()) == 3 << 20
