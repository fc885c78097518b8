"""Can the RCCL data plane (parallel.p2p over a 2-rank nccl pair group, side HIP stream) execute on a
ONE-GPU box, both ranks on device 0?  Launch:
  python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 scripts/exp/rccl_same_gpu.py
Rank 0 ships token ids to rank 1 and back, then times 4 KiB pings; one JSON line per rank."""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from distributed_llm_amd.parallel import p2p  # noqa: E402


def main():
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    dist.init_process_group("nccl")
    pair = dist.new_group([0, 1])
    out = {"rank": rank, "backend": dist.get_backend(pair)}
    try:
        ids = list(range(1000, 1000 + 257))
        if rank == 0:
            p2p.send_tokens(ids, 1, pair, timeout_s=30)
            back = p2p.recv_tokens(1, pair, timeout_s=30).tolist()
            out["roundtrip_ok"] = back == [i + 1 for i in ids]
            out["ping_us"] = [round(p2p.ping(1, pair, initiator=True, timeout_s=30), 1) for _ in range(5)]
        else:
            got = p2p.recv_tokens(0, pair, timeout_s=30).tolist()
            p2p.send_tokens([i + 1 for i in got], 0, pair, timeout_s=30)
            for _ in range(5):
                p2p.ping(0, pair, initiator=False, timeout_s=30)
        out["side_stream"] = str(p2p.side_stream(torch.device("cuda", 0)))
    except Exception as e:  # noqa: BLE001 - reported, not hidden
        out["error"] = f"{type(e).__name__}: {e}"[:400]
    out["s"] = round(time.perf_counter() - t0, 2)
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
