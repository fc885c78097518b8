"""bench.py with the prefill buckets autotuned (ops.gemm.PREFILL_TUNE): the fused ops' core per
(2K / 4K / 8K rows, N, K) chosen between tgemm (64- and 32-deep plans, epilogue fused) and
hipBLASLt + the standalone epilogue.  Same argv as bench.py; an A/B against the default (vendor
prefill core) on one box."""
import os
import runpy
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from distributed_llm_amd.ops import gemm as G  # noqa: E402

G.PREFILL_TUNE = True
sys.argv = [os.path.join(os.path.dirname(__file__), "..", "..", "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
