"""bench.py with class / module constants overridden, for same-box A/B runs of a default:
    python scripts/exp/bench_ab.py engine.KV_PLACEMENT=1 gemm.PREFILL_TUNE=1 -- --steps 20 --warmup 5
``engine.X`` sets LLMEngine.X, ``gemm.X`` sets distributed_llm_amd.ops.gemm.X (ints; 0/1 for flags).
Everything after ``--`` goes to bench.py."""
import os
import runpy
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
from distributed_llm_amd.engine.llm_engine import LLMEngine  # noqa: E402
from distributed_llm_amd.ops import gemm as G  # noqa: E402

args = sys.argv[1:]
cut = args.index("--") if "--" in args else len(args)
for kv in args[:cut]:
    k, v = kv.split("=", 1)
    scope, name = k.split(".", 1)
    target = {"engine": LLMEngine, "gemm": G}[scope]
    old = getattr(target, name)
    setattr(target, name, type(old)(int(v)) if isinstance(old, (bool, int)) else type(old)(v))
    print(f"bench_ab: {k} = {getattr(target, name)!r}", flush=True)
sys.argv = [os.path.join(ROOT, "bench.py")] + args[cut + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
