"""Model architecture registry (public config facts of the BASELINE.json model families).

SURVEY §2.4 op inventory lists the shapes; BASELINE.json configs name TinyLlama-1.1B,
Llama-3.2-1B, Llama-3-8B, Llama-3-70B, Mixtral-8x7B; the reference's own tiers ran
phi3-mini (Nano) and llama3-8B (Orin) under Ollama (src/devices/nano_api.py:16,
src/devices/orin_api.py:18).
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Dict, Optional


@dataclass(frozen=True)
class ModelConfig:
    name: str
    hidden: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    head_dim: int
    intermediate: int
    vocab: int
    rope_theta: float = 10000.0
    rms_eps: float = 1e-5
    max_position: int = 8192
    tie_embeddings: bool = False
    n_experts: int = 0          # > 0: MoE MLP (Mixtral)
    experts_per_token: int = 2
    rope_scaling: Optional[Dict] = None
    bos_id: int = 1
    eos_id: int = 2

    @property
    def is_moe(self) -> bool:
        return self.n_experts > 0

    @property
    def q_size(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.n_kv_heads * self.head_dim

    def num_params(self) -> int:
        H, I, L, V = self.hidden, self.intermediate, self.n_layers, self.vocab
        attn = H * (self.q_size + 2 * self.kv_size) + self.q_size * H
        mlp = 3 * H * I * (self.n_experts if self.is_moe else 1) + (H * self.n_experts if self.is_moe else 0)
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + 2 * H) + emb + H


_LLAMA3_SCALING = {"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                   "original_max_position_embeddings": 8192}

MODELS: Dict[str, ModelConfig] = {
    "tinyllama-1.1b": ModelConfig("tinyllama-1.1b", 2048, 22, 32, 4, 64, 5632, 32000, 10000.0, 1e-5, 16384),
    "llama-3.2-1b": ModelConfig("llama-3.2-1b", 2048, 16, 32, 8, 64, 8192, 128256, 500000.0, 1e-5, 131072,
                                tie_embeddings=True, rope_scaling=_LLAMA3_SCALING, bos_id=128000, eos_id=128001),
    "llama-3-8b": ModelConfig("llama-3-8b", 4096, 32, 32, 8, 128, 14336, 128256, 500000.0, 1e-5, 16384,
                              bos_id=128000, eos_id=128001),
    "llama-3-70b": ModelConfig("llama-3-70b", 8192, 80, 64, 8, 128, 28672, 128256, 500000.0, 1e-5, 16384,
                               bos_id=128000, eos_id=128001),
    "phi3-mini": ModelConfig("phi3-mini", 3072, 32, 32, 32, 96, 8192, 32064, 10000.0, 1e-5, 8192),
    "mixtral-8x7b": ModelConfig("mixtral-8x7b", 4096, 32, 32, 8, 128, 14336, 32000, 1e6, 1e-5, 32768,
                                n_experts=8, experts_per_token=2),
    # small shapes for CPU tests / smoke runs (same code paths)
    "tiny-llama-test": ModelConfig("tiny-llama-test", 128, 2, 4, 2, 32 * 2, 256, 512, 10000.0, 1e-5, 2048),
    "tiny-moe-test": ModelConfig("tiny-moe-test", 128, 2, 4, 2, 64, 128, 512, 10000.0, 1e-5, 2048,
                                 n_experts=4, experts_per_token=2),
}

ALIASES = {"tinyllama": "tinyllama-1.1b", "llama3-1b": "llama-3.2-1b", "llama3-8b": "llama-3-8b",
           "llama3": "llama-3-8b", "llama3-70b": "llama-3-70b", "phi3": "phi3-mini", "mixtral": "mixtral-8x7b"}


def get_model_config(name: str, **overrides) -> ModelConfig:
    key = ALIASES.get(name.lower(), name.lower())
    if key not in MODELS:
        raise KeyError(f"unknown model {name!r}; known: {sorted(MODELS)}")
    cfg = MODELS[key]
    return replace(cfg, **overrides) if overrides else cfg
