"""Worker for tests/test_custom_ar_gpu.py: one rank of a 2-rank group sharing ONE GPU.

The one-shot all-reduce only needs IPC-mappable peer memory, which works between processes on
the same device, so the protocol (copy, flags, double buffering, graph replay) is exercised on a
1-GPU box; the 8-GPU xGMI case uses the identical code path.
"""
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, sys.argv[4])
from distributed_llm_amd.parallel.custom_ar import CustomAllReduce  # noqa: E402


def inputs(rank, n, salt=0):
    g = torch.Generator().manual_seed(1000 * n + 17 * rank + salt)
    return torch.randn(n, generator=g).to(torch.bfloat16)


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    car = CustomAllReduce(dist.group.WORLD, torch.device("cuda:0"), max_bytes=1 << 20)
    fails = []
    for n in (8, 64, 1024, 2048 * 3, 16384 + 8, 262144, 524288):
        want = sum(inputs(r, n).float() for r in range(world)).to(torch.bfloat16)
        x = inputs(rank, n).cuda()
        assert car.eligible(x)
        out = torch.empty_like(x)
        car.all_reduce(x, out)          # out of place
        car.all_reduce(x)               # in place
        torch.cuda.synchronize()
        for name, got in (("out", out), ("inplace", x)):
            if not torch.equal(got.cpu(), want):
                fails.append(f"n={n} {name}: max err {(got.cpu().float() - want.float()).abs().max().item()}")
    # captured in a hipGraph: the epoch advances on the device across replays
    n = 2048 * 8
    xs = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        car.all_reduce(xs)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        car.all_reduce(xs)
    for it in range(6):
        xs.copy_(inputs(rank, n, salt=it + 1).cuda())
        g.replay()
        torch.cuda.synchronize()
        want = sum(inputs(r, n, salt=it + 1).float() for r in range(world)).to(torch.bfloat16)
        if not torch.equal(xs.cpu(), want):
            fails.append(f"graph replay {it}")
    car.check()
    # a peer that never arrives: rank 1 skips one all-reduce while rank 0 spins out (bounded);
    # the error flag trips on rank 0 only, and the consensus check drops the custom all-reduce on
    # BOTH ranks (ParallelContext.check_collectives), so neither deadlocks nor diverges
    from distributed_llm_amd.parallel.comm import ParallelContext
    par = ParallelContext(tp_size=world, tp_rank=rank, tp_group=dist.group.WORLD, global_rank=rank,
                          world_size=world, custom_ar=car)
    assert par.check_collectives()
    dist.barrier()
    car.spin_limit = 20000
    if rank == 0:
        y = inputs(rank, 4096).cuda()
        car.all_reduce(y)
        torch.cuda.synchronize()
    dist.barrier()
    tripped = not par.check_collectives()
    if not tripped or par.custom_ar is not None:
        fails.append(f"rank {rank}: timeout not agreed (tripped={tripped})")
    dist.barrier()
    car.close()
    dist.destroy_process_group()
    if fails:
        print("FAIL", fails, flush=True)
        sys.exit(1)
    print("OK", flush=True)


if __name__ == "__main__":
    main()
