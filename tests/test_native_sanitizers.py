"""Race / memory checking (the reference has none).

* Native runtime: the paged-KV block manager core (csrc/runtime/block_manager.h) is driven by a
  randomised stress program (csrc/runtime/tests/block_manager_stress.cpp) built with
  AddressSanitizer + UndefinedBehaviorSanitizer on the host; it checks structural invariants and
  KV-slot contents after every operation (prefix re-use, eviction, preemption).
* The Python binding exposes the same invariant check; it is run after a CPU engine workload.
GPU sanitizers are not available on the MI355X pool, so kernels are covered by the numerics and
resource (no scratch) tests instead.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "runtime", "tests", "block_manager_stress.cpp")


def _build(tmp_path_factory, name, extra):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    out = str(tmp_path_factory.mktemp("asan") / name)
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-Wall", "-Werror", *extra, SRC, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return out


@pytest.fixture(scope="module")
def asan_binary(tmp_path_factory):
    return _build(tmp_path_factory, "block_manager_stress", [])


@pytest.fixture(scope="module")
def asan_weak_hash_binary(tmp_path_factory):
    # 3-bit chain hash: almost every lookup collides, so only the stored-token check keeps a
    # prefix-cache hit from handing out another sequence's K/V (block_manager.h)
    return _build(tmp_path_factory, "block_manager_stress_weak", ["-DDLLM_BM_WEAK_HASH"])


def _run(binary, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([binary, "20000", str(seed)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok "), r.stdout
    assert "runtime error" not in r.stderr  # UBSan report
    return r.stdout


@pytest.mark.parametrize("seed", [1, 7, 2024])
def test_block_manager_stress_under_asan_ubsan(asan_binary, seed):
    _run(asan_binary, seed)


@pytest.mark.parametrize("seed", [3, 11])
def test_block_manager_forced_hash_collisions(asan_weak_hash_binary, seed):
    out = _run(asan_weak_hash_binary, seed)
    assert "collisions=" in out and " collisions=0 " not in out + " ", out


def test_binding_invariants_after_engine_workload():
    from distributed_llm_amd.engine.llm_engine import LLMEngine
    from distributed_llm_amd.engine.sampling import SamplingParams

    eng = LLMEngine("tiny-llama-test", device="cpu", kv_cache_gb=0.01, max_num_seqs=8, seed=0)
    sp = SamplingParams(max_new_tokens=20, temperature=0.0, ignore_eos=True)
    base = [f"user: conversation {i} " + "word " * (10 + 7 * i) for i in range(6)]
    outs = eng.generate(base, sp)
    # second turn of each conversation: the prefix blocks are matched again
    outs = eng.generate([b + o.text + "\nuser: more" for b, o in zip(base, outs)], sp)
    assert all(o.error is None for o in outs)
    assert eng.bm.check_invariants() == ""
    st = eng.bm.stats()
    assert st["active_seqs"] == 0 and st["prefix_hit_tokens"] > 0
