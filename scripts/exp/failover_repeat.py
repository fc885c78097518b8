"""Run the config-4 leader-death rehearsal N times in one process and keep the logs of any run
whose exit codes differ from (rank 4: 17, others: 0) (diagnosing an intermittent rank-0 exit)."""
import os
import shutil
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests import test_pools_gpu as T  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
base = "gpurun_out/failover_repeat"
for i in range(n):
    d = os.path.join(base, f"run{i}")
    os.makedirs(d, exist_ok=True)
    print(f"run {i} ...", flush=True)
    try:
        codes, res, logs = T._launch_ranks(8, ["--baseline-config", "4", *T.SMALL_RUN], d, "cfg4fo",
                                           {"DLLM_FAULT": "die_rank=4,die_after=2", "DLLM_STACK_DUMP_S": "75"},
                                           timeout=120)
    except subprocess.TimeoutExpired:
        print(f"run {i}: HUNG (logs kept in {d})", flush=True)
        break
    ok = codes[4] == 17 and all(c == 0 for j, c in enumerate(codes) if j != 4)
    print(f"run {i}: codes {codes} {'ok' if ok else 'BAD'}", flush=True)
    if ok:
        shutil.rmtree(d)
