"""Token counting for routing decisions and response metrics.

Reference: ``src/token_counter.py:4-12`` (litellm, model "ollama/phi3") and the token
router's count at ``src/query_router_engine.py:93-96`` (litellm, else ``len//4``).

litellm is not part of this stack.  Counting order:
  1. a real ``tokenizers`` tokenizer if a ``tokenizer.json`` path is configured
     (``DLLM_TOKENIZER`` env or ``set_tokenizer_path``);
  2. the reference's own fallback ``max(1, len(text) // 4)``.
Message lists add a fixed 3-token per-message frame, like chat templates do
(litellm's exact framing is model specific — parity unpinned, documented in tests).
"""
from __future__ import annotations

import os
import threading
from typing import Dict, Iterable, List, Optional

_lock = threading.Lock()
_tok = None
_tok_path: Optional[str] = None


def set_tokenizer_path(path: Optional[str]) -> None:
    global _tok, _tok_path
    with _lock:
        _tok_path = path
        _tok = None


def _get_tokenizer():
    global _tok, _tok_path
    if _tok is not None:
        return _tok
    path = _tok_path or os.environ.get("DLLM_TOKENIZER")
    if not path or not os.path.exists(path):
        return None
    with _lock:
        if _tok is None:
            from tokenizers import Tokenizer
            _tok = Tokenizer.from_file(path)
    return _tok


def count_text(text: str) -> int:
    tok = _get_tokenizer()
    if tok is not None:
        return len(tok.encode(text or "").ids)
    return max(1, len(text or "") // 4)


MESSAGE_FRAME_TOKENS = 3


def count_messages(messages: Iterable[Dict[str, str]]) -> int:
    total = 0
    for m in messages:
        if not isinstance(m, dict):
            continue
        total += MESSAGE_FRAME_TOKENS + count_text(str(m.get("content") or ""))
    return total


class TokenCounter:
    """Drop-in for the reference ``TokenCounter`` (``src/token_counter.py``)."""

    def count_tokens(self, msg: Dict[str, str]) -> int:
        return count_messages([msg])

    def get_context_size(self, context: List[Dict[str, str]]) -> int:
        return count_messages(context)
