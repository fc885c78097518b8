"""Interactive chat REPL (reference ``src/main.py:3-27``).

``You:`` prompt -> ``Router.route_query(history)``; ``exit``/``quit`` stops the pools' servers.
Prints the reply followed by the response token count, like the reference.

Run: ``python -m distributed_llm_amd.server.cli --strategy semantic [--pools echo|gpu]``
"""
from __future__ import annotations

import argparse
import sys
from typing import Any, Dict, Optional


class Chatbot:
    def __init__(self, strategy: str = "token", config: Optional[Dict[str, Any]] = None, threshold_fallback: int = 100,
                 pools=None):
        from ..orchestrator import Router
        self.router = Router(strategy=strategy, config=config or {}, threshold_fallback=threshold_fallback,
                             pools=pools)
        self.conversation_history = []

    def add_message(self, role: str, content: str) -> None:
        self.conversation_history.append({"role": role, "content": content})

    def turn(self, text: str):
        self.add_message("user", text)
        resp, ntok, dev = self.router.route_query(self.conversation_history)
        reply = resp.get("response", "") if isinstance(resp, dict) else str(resp)
        self.add_message("assistant", reply)
        return reply, ntok, dev

    def chat(self, stdin=sys.stdin, stdout=sys.stdout) -> None:
        while True:
            stdout.write("You: ")
            stdout.flush()
            line = stdin.readline()
            if not line:
                break
            text = line.rstrip("\n")
            if text.lower() in ("exit", "quit"):
                self.router.orin.server_manager.stop_server()
                self.router.nano.server_manager.stop_server()
                break
            reply, ntok, _dev = self.turn(text)
            stdout.write(f"Assistant: {reply} {ntok}\n")


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--strategy", default="semantic")
    ap.add_argument("--pools", default="echo")
    ap.add_argument("--model", default="tinyllama-1.1b")
    a = ap.parse_args(argv)
    from ..bench.harness import build_pools_from_arg
    pools, _, _ = build_pools_from_arg(a.pools, a.model, None, None)
    Chatbot(strategy=a.strategy, config={"cache_enabled": False, "enable_response_cache": False,
                                         "enable_failover": True}, pools=pools).chat()


if __name__ == "__main__":
    main()
