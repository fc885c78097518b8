"""Host HTTP API — byte-compatible ``/chat`` and ``/history`` (reference ``src/app.py``).

Reference: POST /chat :27-106, GET /history :109-113, DELETE /history :116-121, base config
:9-14, history cap :23.  Same request/response JSON, status codes and history semantics
(user turn appended before routing and rolled back on error; last 10 messages kept).
Differences: state is lock-protected (the reference mutates module globals from Flask's threaded
server), CORS headers are set without flask-cors, and ``GET /metrics`` exposes cache statistics,
pool health, engine counters and the last reply's timing.  A ``/chat`` reply carries exactly the
reference's seven keys (``src/app.py:83-91`` and ``:98-106``); a client that sends
``"include_timing": true`` (the bundled UI does) gets an eighth, ``timing``; ``GET /`` serves a no-build browser chat client with the same
request/metadata contract as the reference React app (server/static/index.html).

Run:  ``python -m distributed_llm_amd.server.app --pools echo|gpu [--port 8000]``
"""
from __future__ import annotations

import argparse
import threading
from typing import Any, Dict, List, Optional

import os

from flask import Flask, jsonify, request, send_from_directory

from ..config import CLASS_DEFAULTS

HISTORY_LIMIT = 10
_STATIC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "static")

BASE_CONFIG: Dict[str, Any] = {
    "cache_enabled": True,
    "enable_response_cache": True,
    "enable_failover": True,
    "weights": {"token": 0.25, "semantic": 0.45, "heuristic": 0.30},
}

STRATEGY_ALIASES = {"token-counting": "token"}


def create_app(router=None, config: Optional[Dict[str, Any]] = None, pools=None) -> Flask:
    from ..orchestrator import Router
    app = Flask(__name__)
    state = {
        "router": router or Router(strategy="hybrid", config=dict(config or BASE_CONFIG), pools=pools),
        "strategy": "hybrid",
        "histories": {},
    }
    if router is not None:
        state["strategy"] = router.query_router.strategy
    lock = threading.RLock()

    @app.after_request
    def _cors(resp):
        resp.headers["Access-Control-Allow-Origin"] = "*"
        resp.headers["Access-Control-Allow-Headers"] = "Content-Type"
        resp.headers["Access-Control-Allow-Methods"] = "GET, POST, DELETE, OPTIONS"
        return resp

    @app.route("/chat", methods=["POST", "OPTIONS"])
    def chat():
        if request.method == "OPTIONS":
            return "", 204
        data = request.get_json(silent=True) or {}
        message = data.get("message", "")
        strategy = STRATEGY_ALIASES.get(data.get("strategy", "hybrid"), data.get("strategy", "hybrid"))
        session = data.get("session_id", "default")
        want_timing = data.get("include_timing") is True   # opt-in: the reference contract has 7 keys
        if not isinstance(message, str) or not message.strip():
            return jsonify({"error": "No message provided"}), 400
        r = state["router"]
        with lock:
            if strategy != state["strategy"]:
                try:
                    r.query_router.change_strategy(strategy)
                    state["strategy"] = strategy
                except Exception as e:
                    return jsonify({"error": f"Failed to switch strategy: {e}"}), 500
            hist: List[Dict[str, str]] = state["histories"].setdefault(session, [])
            hist.append({"role": "user", "content": message})
            snapshot = list(hist)
        try:
            payload, tokens, device = r.route_query(snapshot)
            timing: Dict[str, Any] = {}
            if isinstance(payload, dict):
                reply = payload.get("response", "")
                reasoning = payload.get("routing_reasoning", f"Method: {strategy}")
                method = payload.get("routing_method", strategy)
                confidence = payload.get("routing_confidence", 0.0)
                cache_hit = payload.get("cache_hit", False)
                raw = payload.get("raw") if isinstance(payload.get("raw"), dict) else {}
                # extra keys for the metadata panel (reference clients ignore unknown keys)
                timing = {"latency_ms": raw.get("latency_ms"), "routing_ms": payload.get("routing_overhead_ms"),
                          "ttft_ms": (payload.get("timing") or {}).get("ttft_ms"),
                          "failover": bool(payload.get("failover") or raw.get("failover"))}
            else:
                reply, reasoning, method, confidence, cache_hit = str(payload), "Direct response", strategy, 0.0, False
            with lock:
                hist = state["histories"].setdefault(session, [])
                hist.append({"role": "assistant", "content": reply})
                state["histories"][session] = hist[-HISTORY_LIMIT:]
                state["last_timing"] = dict(timing, session_id=session)
            body = {"reply": reply, "device": device, "reasoning": reasoning, "method": method,
                    "confidence": confidence, "cache_hit": cache_hit, "tokens": tokens}
            if want_timing:
                body["timing"] = timing
            return jsonify(body)
        except Exception as e:
            with lock:
                hist = state["histories"].get(session, [])
                if hist and hist[-1]["role"] == "user":
                    hist.pop()
            body = {"reply": "System Error: The router encountered an issue.", "device": "error",
                    "reasoning": str(e), "method": strategy, "confidence": 0.0, "cache_hit": False, "tokens": 0}
            if want_timing:
                body["timing"] = {}
            return jsonify(body), 500

    @app.route("/", methods=["GET"])
    def ui():
        """Browser chat client (server/static/index.html; reference fyp-chat-frontend App.tsx)."""
        return send_from_directory(_STATIC, "index.html")

    @app.route("/history", methods=["GET"])
    def get_history():
        sid = request.args.get("session_id", "default")
        with lock:
            return jsonify(list(state["histories"].get(sid, [])))

    @app.route("/history", methods=["DELETE"])
    def clear_history():
        sid = request.args.get("session_id", "default")
        with lock:
            state["histories"].pop(sid, None)
        return jsonify({"cleared": sid})

    @app.route("/metrics", methods=["GET"])
    def metrics():
        r = state["router"]
        pools = {name: _safe(p.health) for name, p in r.pools.items()}
        return jsonify({"strategy": state["strategy"], "cache": r.query_router.get_cache_stats(), "pools": pools,
                        "sessions": len(state["histories"]), "last_timing": state.get("last_timing")})

    app.config["DLLM_STATE"] = state
    return app


def _safe(fn):
    try:
        return fn()
    except Exception as e:  # health must never take the API down
        return {"ok": False, "error": str(e)}


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--pools", default="echo", help="echo | gpu | path to a JSON/YAML pool topology")
    ap.add_argument("--model", default="tinyllama-1.1b")
    a = ap.parse_args(argv)
    cfg = dict(BASE_CONFIG)
    if a.pools == "gpu":
        cfg["pools"] = {"nano": {"model": a.model, "max_new_tokens": 128, "share": "main"},
                        "orin": {"model": a.model, "max_new_tokens": 384, "temperature": 0.8, "top_k": 40,
                                 "top_p": 0.9, "share": "main"}}
    elif a.pools != "echo":
        from ..config import load_config_file
        cfg["pools"] = load_config_file(a.pools)
    app = create_app(config=cfg)
    print(f"API running on http://{a.host}:{a.port}")
    app.run(host=a.host, port=a.port, threaded=True)


if __name__ == "__main__":
    main()
