"""Pool-worker HTTP shim — the reference device API (``src/devices/nano_api.py``,
``src/devices/orin_api.py``) served in front of OUR engine instead of Ollama.

Endpoints (same contract):  ``GET /`` -> "Test again: Server is running!\\n";
``GET /health`` -> ``{"ok": true}``;  ``POST /query {"query": list|str, "num_predict"?,
"temperature"?, "top_k"?, "top_p"?}`` -> ``{"response": str}`` | 400/504/500 ``{"error": ...}``.
Additions: ``POST /query {"queries": [...]}`` serves a batch (continuous batching) and returns
``{"responses": [...]}``; responses carry ``num_tokens`` and timing.

One worker process owns one pool = a GPU subset (``HIP_VISIBLE_DEVICES`` set by the supervisor)
and, for tp > 1, one process per GPU under torchrun with rank 0 serving HTTP.
"""
from __future__ import annotations

import argparse
import logging
import threading
from typing import Any, Dict

from flask import Flask, jsonify, request

from .base import EchoPool, EnginePool, PoolClient, format_prompt

log = logging.getLogger("dllm.pool")


def create_worker_app(pool: PoolClient) -> Flask:
    app = Flask(__name__)
    lock = threading.Lock()

    @app.route("/")
    def home():
        return "Test again: Server is running!\n", 200

    @app.route("/health", methods=["GET"])
    def health():
        return jsonify({"ok": True}), 200

    @app.route("/stats", methods=["GET"])
    def stats():
        return jsonify(pool.health())

    def _overrides(data: Dict[str, Any]) -> Dict[str, Any]:
        return {k: data[k] for k in ("num_predict", "temperature", "top_k", "top_p") if k in data}

    @app.route("/query", methods=["POST"])
    def query():
        data = request.get_json(silent=True) or {}
        if "queries" in data:
            qs = data.get("queries") or []
            if not isinstance(qs, list) or not qs:
                return jsonify({"error": "No query provided"}), 400
            try:
                if isinstance(pool, EnginePool):
                    res = pool.process_batch(qs, _overrides(data))
                else:
                    res = pool.process_batch(qs)
                return jsonify({"responses": res})
            except Exception as e:
                return jsonify({"error": f"engine failed: {e}"}), 500
        q = data.get("query")
        if not q:
            return jsonify({"error": "No query provided"}), 400
        if not isinstance(q, (list, str)):
            return jsonify({"error": "Invalid query format. Expect list[role/content] or string."}), 400
        if not format_prompt(q):
            return jsonify({"error": "Empty query after formatting."}), 400
        try:
            with lock if not isinstance(pool, EnginePool) else _nolock:
                res = pool.process(q, _overrides(data)) if isinstance(pool, EnginePool) else pool.process(q)
        except TimeoutError:
            return jsonify({"error": "engine timed out"}), 504
        except Exception as e:
            return jsonify({"error": f"engine failed: {e}"}), 500
        if "error" in res:
            return jsonify(res), 500
        return jsonify(res)

    return app


class _NoLock:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


_nolock = _NoLock()


def _tp_setup(a):
    """Under torchrun (WORLD_SIZE > 1): one process per GPU of the pool, bound to LOCAL_RANK; all
    ranks form ONE tensor-parallel group (RCCL on GPU, gloo on CPU) plus a gloo group for the
    scheduler mirror.  Returns (ParallelContext, mirror group, device)."""
    import os
    import torch
    import torch.distributed as dist
    from ..parallel.comm import init_distributed, make_tp_groups
    local = int(os.environ.get("LOCAL_RANK", "0"))
    on_gpu = a.device == "cuda" and torch.cuda.is_available()
    if on_gpu:
        torch.cuda.set_device(local)
    init_distributed("nccl" if on_gpu else "gloo")
    par = make_tp_groups(dist.get_world_size())
    mirror = dist.new_group(list(range(dist.get_world_size())), backend="gloo")
    dev = f"cuda:{local}" if on_gpu else "cpu"
    if on_gpu:
        par.enable_custom_all_reduce(dev)
    return par, mirror, dev


def main(argv=None) -> None:
    import os
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", default="nano")
    ap.add_argument("--port", type=int, default=5001)
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--kind", default="engine", choices=["engine", "echo"])
    ap.add_argument("--model", default="tinyllama-1.1b")
    ap.add_argument("--max-new-tokens", type=int, default=256)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--kv-gb", type=float, default=None)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    a = ap.parse_args(argv)
    if a.kind == "echo":
        pool: PoolClient = EchoPool(a.name, tokens_per_reply=min(a.max_new_tokens, 64))
        create_worker_app(pool).run(host=a.host, port=a.port, threaded=True)
        return
    from ..engine.llm_engine import LLMEngine
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # tensor-parallel pool (supervisor launches torchrun, one rank per GPU): rank 0 serves HTTP
        # and leads the scheduler; the other ranks replay it in lockstep (LLMEngine.follow)
        import torch.distributed as dist
        par, mirror, dev = _tp_setup(a)
        eng = LLMEngine(a.model, device=dev, par=par, kv_cache_gb=a.kv_gb, max_num_seqs=a.max_num_seqs)
        eng.enable_tp_mirror(mirror, 0)
        if dist.get_rank() != 0:
            eng.follow()
            return
        eng.start()
        pool = EnginePool(a.name, eng, max_new_tokens=a.max_new_tokens, temperature=a.temperature)
        try:
            create_worker_app(pool).run(host=a.host, port=a.port, threaded=True)
        finally:
            eng.stop()   # members leave follow()
        return
    dev = a.device
    eng = LLMEngine(a.model, device=dev, kv_cache_gb=a.kv_gb, max_num_seqs=a.max_num_seqs)
    eng.start()
    pool = EnginePool(a.name, eng, max_new_tokens=a.max_new_tokens, temperature=a.temperature)
    create_worker_app(pool).run(host=a.host, port=a.port, threaded=True)


if __name__ == "__main__":
    main()
