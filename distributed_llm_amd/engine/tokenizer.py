"""Tokenizers.

No model checkpoints or vocab files exist in this environment, so the default is a
deterministic byte-level tokenizer (prefix-stable: a conversation's previous turn tokenises to
a prefix of the next turn's prompt, which is what lets the prefix cache reuse KV blocks).
A HF ``tokenizer.json`` is used when given (``tokenizers`` library).
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np


class ByteTokenizer:
    """ids: 0 pad, 1 bos, 2 eos, 3..258 = bytes; ids >= 259 (random-weight models emit them)
    decode to printable ASCII so generated text round-trips through the conversation."""

    OFFSET = 3

    def __init__(self, vocab_size: int, bos_id: int = 1, eos_id: int = 2):
        if vocab_size < 259:
            raise ValueError("byte tokenizer needs vocab >= 259")
        self.vocab_size = vocab_size
        self.bos_id = bos_id if bos_id < vocab_size else 1
        self.eos_id = eos_id if eos_id < vocab_size else 2

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = (np.frombuffer(text.encode("utf-8"), dtype=np.uint8).astype(np.int64) + self.OFFSET).tolist()
        return ([self.bos_id] + ids) if add_bos else ids

    def decode(self, ids) -> str:
        a = np.asarray(ids, dtype=np.int64).reshape(-1)
        a = a[(a >= self.OFFSET) & (a != self.bos_id) & (a != self.eos_id)]
        b = np.where(a < 256 + self.OFFSET, a - self.OFFSET, 32 + a % 95).astype(np.uint8)
        return b.tobytes().decode("utf-8", errors="replace")


class HFTokenizer:
    def __init__(self, path: str, bos_id: Optional[int] = None, eos_id: Optional[int] = None):
        from tokenizers import Tokenizer
        self.tok = Tokenizer.from_file(path)
        self.vocab_size = self.tok.get_vocab_size()
        self.bos_id = bos_id if bos_id is not None else 1
        self.eos_id = eos_id if eos_id is not None else 2

    def encode(self, text: str, add_bos: bool = True) -> List[int]:
        ids = self.tok.encode(text, add_special_tokens=False).ids
        return ([self.bos_id] + ids) if add_bos else ids

    def decode(self, ids) -> str:
        return self.tok.decode([int(i) for i in ids], skip_special_tokens=True)


def get_tokenizer(vocab_size: int, bos_id: int, eos_id: int, path: Optional[str] = None):
    path = path or os.environ.get("DLLM_TOKENIZER")
    if path and os.path.exists(path):
        return HFTokenizer(path, bos_id, eos_id)
    return ByteTokenizer(vocab_size, bos_id, eos_id)
