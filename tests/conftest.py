import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels on cuda:0)")
    config.addinivalue_line("markers", "slow: multi-process / long tests")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session", autouse=True)
def _native_runtime():
    """Build the C++ runtime (g++, seconds) if it is missing; the HIP kernels are built by
    __graft_entry__.build() / `python -m distributed_llm_amd._build`."""
    from distributed_llm_amd import _build
    _build.build_runtime(force=False)
    yield


@pytest.fixture(autouse=True)
def _hash_embedder(monkeypatch):
    # CPU tests use the deterministic hashing embedder unless a test opts out
    if not os.environ.get("DLLM_EMBEDDER"):
        monkeypatch.setenv("DLLM_EMBEDDER", "hash")
    from distributed_llm_amd.router import embedder
    embedder.clear_registry()
    yield
