"""One-shot IPC all-reduce (csrc/kernels/custom_ar.hip) vs an exact f32 reference sum.

Two ranks share the single GPU of the test box (IPC mapping works within one device), each a
separate process started with subprocess (gloo only exchanges the IPC handles)."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_custom_all_reduce_two_ranks_one_gpu():
    port, world = _port(), 2
    worker = os.path.join(ROOT, "tests", "workers", "custom_ar_worker.py")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, worker, str(r), str(world), str(port), ROOT], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=300)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rc, out in outs:
        assert rc == 0 and "OK" in out, out[-3000:]
