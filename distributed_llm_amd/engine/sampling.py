"""Sampling parameters.

Reference defaults: the small tier decodes greedily (``temperature=0.0``, ``num_predict=-1``
i.e. until EOS; src/devices/nano_api.py:20-21); the large tier uses Ollama's defaults
(src/devices/orin_api.py:57-61: temperature 0.8, top_k 40, top_p 0.9 — [ext] Ollama docs).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass


@dataclass
class SamplingParams:
    max_new_tokens: int = 256
    temperature: float = 0.0      # 0 -> greedy
    top_k: int = 0                # 0 -> no top-k cut (nucleus over the top CANDIDATES logits)
    top_p: float = 1.0
    ignore_eos: bool = False
    seed: int = 0

    CANDIDATES = 256              # width of the candidate set for sampled decoding

    @property
    def greedy(self) -> bool:
        return self.temperature <= 0.0

    @property
    def k(self) -> int:
        return self.top_k if self.top_k > 0 else self.CANDIDATES

    def to_dict(self) -> dict:
        return asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "SamplingParams":
        return cls(**{k: v for k, v in d.items() if k in cls.__dataclass_fields__})


OLLAMA_DEFAULTS = SamplingParams(max_new_tokens=256, temperature=0.8, top_k=40, top_p=0.9)
GREEDY = SamplingParams(max_new_tokens=256, temperature=0.0)
