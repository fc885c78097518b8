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
    # fused residual add + row statistics (car_resadd) and the one-shot all-gather
    for T, H in ((1, 2048), (5, 4096), (64, 8192), (37, 3072), (3, 64)):
        ys = [inputs(r, T * H, salt=7).view(T, H) for r in range(world)]
        r0 = inputs(99, T * H, salt=3).view(T, H)
        tot = sum(y.float() for y in ys).to(torch.bfloat16)           # all-reduce output (bf16)
        for add in (True, False):
            want = (tot.float() + r0.float()).to(torch.bfloat16) if add else tot
            rr = r0.clone().cuda()
            ssq = torch.full((40, T), -1.0, device="cuda")
            n = car.all_reduce_resadd(ys[rank].cuda(), rr, ssq, add)
            torch.cuda.synchronize()
            if not torch.equal(rr.cpu(), want):
                fails.append(f"resadd T={T} H={H} add={add}: max err {(rr.cpu().float() - want.float()).abs().max()}")
            got = ssq[:n].sum(0).cpu()
            ref = want.float().pow(2).sum(1)
            if not torch.allclose(got, ref, rtol=1e-4, atol=1e-3) or n != car.resadd_slots(H):
                fails.append(f"resadd ssq T={T} H={H} n={n}")
    for n in (8, 256 * 3, 8 * 512):
        x = inputs(rank, n, salt=11).cuda()
        got = car.all_gather(x)
        torch.cuda.synchronize()
        want = torch.stack([inputs(r, n, salt=11) for r in range(world)])
        if not torch.equal(got.cpu(), want):
            fails.append(f"all_gather n={n}")
    xi = torch.arange(64, dtype=torch.int32, device="cuda") + 1000 * rank
    gi = car.all_gather(xi).cpu()
    if not torch.equal(gi, torch.stack([torch.arange(64, dtype=torch.int32) + 1000 * r for r in range(world)])):
        fails.append("all_gather int32")
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
