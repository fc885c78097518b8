"""Routing/serving configuration profiles.

Key names and default values mirror the reference so configs are interchangeable:
  * ``BENCHMARK_CFG`` / ``PRODUCTION_CFG``  — reference ``src/query_router_engine.py:704-731``
  * ``default_config()``                   — reference ``src/query_router_engine.py:517-553``
  * orchestrator keys (``enable_response_cache``, ``enable_failover``, ``cache_last_k``)
                                           — reference ``src/router.py:45-54``

Reference semantics: a non-empty config dict *replaces* the defaults (no merge,
``query_router_engine.py:487``).  That behaviour is kept as the default so parity
runs route identically; pass ``merge_defaults=True`` to ``resolve_config`` (or set
``"merge_defaults": True`` in the dict) to layer a partial dict over the defaults.

Pool topology (new): ``pools`` maps a tier name to where/what it serves, e.g.
``{"nano": {"model": "tinyllama-1.1b", "gpus": [0], "tp": 1}, "orin": {...}}``.
"""
from __future__ import annotations

import copy
import json
import os
from typing import Any, Dict, Optional

# Tier names used in every public payload / CSV (reference device names).
SMALL = "nano"
LARGE = "orin"
TIERS = (SMALL, LARGE)
TIER_ALIASES = {"small": SMALL, "nano": SMALL, "large": LARGE, "orin": LARGE}

_DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
DEFAULT_LABEL_PATH = os.path.join(_DATA_DIR, "semantic_labels.json")
QUERY_SET_PATH = os.path.join(_DATA_DIR, "query_sets.json")

BENCHMARK_CFG: Dict[str, Any] = {
    "token_threshold": 1000,
    "model": "meta-llama/Llama-2-7b-hf",
    "embedding_model": "all-MiniLM-L6-v2",
    "semantic_label_path": DEFAULT_LABEL_PATH,
    "semantic_margin_threshold": 0.03,
    "semantic_min_similarity": 0.05,
    "heuristic_long_chars": 800,
    "heuristic_multi_qmarks": 2,
    "heuristic_code_markers_needed": 2,
    "heuristic_context_chars": 3200,
    "weights": {"token": 0.25, "semantic": 0.45, "heuristic": 0.30},
    "cache_enabled": False,
    "perf_window": 30,
    "perf_fail_penalty": 3000.0,
}

PRODUCTION_CFG: Dict[str, Any] = {
    **BENCHMARK_CFG,
    "cache_enabled": True,
    "cache_ttl_seconds": 3600,
    "cache_max_size": 500,
    "cache_similarity_threshold": 0.85,
    "use_semantic_cache": True,
    "prediction_confidence_threshold": 0.70,
    "enable_response_cache": True,
}


def default_config() -> Dict[str, Any]:
    """Config used by QueryRouter when it is given a falsy config."""
    cfg = copy.deepcopy(BENCHMARK_CFG)
    cfg.update({
        "cache_enabled": False,
        "cache_ttl_seconds": 3600,
        "cache_max_size": 500,
        "cache_similarity_threshold": 0.85,
        "use_semantic_cache": True,
        "prediction_confidence_threshold": 0.70,
    })
    return cfg


# Class-level fallbacks (what each component uses when a key is absent).
CLASS_DEFAULTS: Dict[str, Any] = {
    "token_threshold": 1000,
    "model": "meta-llama/Llama-2-7b-hf",
    "embedding_model": "all-MiniLM-L6-v2",
    "semantic_label_path": "",
    "semantic_margin_threshold": 0.03,
    "semantic_min_similarity": 0.05,
    "heuristic_long_chars": 250,
    "heuristic_multi_qmarks": 3,
    "heuristic_code_markers_needed": 2,
    "heuristic_context_chars": 800,
    "weights": {"token": 0.35, "semantic": 0.35, "heuristic": 0.30},
    "cache_enabled": True,
    "cache_ttl_seconds": 3600,
    "cache_max_size": 500,
    "cache_similarity_threshold": 0.85,
    "use_semantic_cache": True,
    "prediction_confidence_threshold": 0.70,
    "perf_window": 30,
    "perf_fail_penalty": 3000.0,
    "enable_response_cache": False,
    "enable_failover": True,
    "cache_last_k": 6,
}


def resolve_config(config: Optional[Dict[str, Any]], merge_defaults: Optional[bool] = None) -> Dict[str, Any]:
    """Return the effective config dict.

    Falsy ``config`` -> ``default_config()`` (reference behaviour).  A non-empty dict is
    used as-is (replace semantics) unless ``merge_defaults`` (argument or key) is true,
    in which case it is layered over ``default_config()``.
    """
    if not config:
        return default_config()
    merge = config.get("merge_defaults", False) if merge_defaults is None else merge_defaults
    if merge:
        out = default_config()
        out.update(config)
        return out
    return config


def load_config_file(path: str) -> Dict[str, Any]:
    """Load a JSON or YAML config (YAML via SafeLoader only)."""
    with open(path, "r", encoding="utf-8") as f:
        text = f.read()
    if path.endswith((".yaml", ".yml")):
        import yaml
        return yaml.load(text, Loader=yaml.SafeLoader) or {}
    return json.loads(text)


def apply_env_overrides(cfg: Dict[str, Any], prefix: str = "DLLM_") -> Dict[str, Any]:
    """Override scalar keys from environment, e.g. ``DLLM_TOKEN_THRESHOLD=500``.

    The reference advertises a ``.env`` config (README.md:77-85) that no code reads;
    this is the working equivalent.
    """
    out = dict(cfg)
    for key, val in os.environ.items():
        if not key.startswith(prefix):
            continue
        name = key[len(prefix):].lower()
        cur = out.get(name, CLASS_DEFAULTS.get(name))
        try:
            if isinstance(cur, bool):
                out[name] = val.lower() in ("1", "true", "yes", "on")
            elif isinstance(cur, int):
                out[name] = int(val)
            elif isinstance(cur, float):
                out[name] = float(val)
            elif isinstance(cur, dict):
                out[name] = json.loads(val)
            else:
                out[name] = val
        except (ValueError, json.JSONDecodeError):
            out[name] = val
    return out


def canonical_tier(name: str) -> str:
    try:
        return TIER_ALIASES[name.lower()]
    except KeyError:
        raise ValueError(f"unknown tier {name!r}; expected one of {sorted(TIER_ALIASES)}") from None


def other_tier(name: str) -> str:
    return LARGE if canonical_tier(name) == SMALL else SMALL
