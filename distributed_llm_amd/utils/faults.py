"""Fault injection for tests and bench diagnostics (``diag``, DLLM_DIAG).

Faults: ONE environment variable,

    DLLM_FAULT="die_after=1,die_rank=2"          (comma-separated key=value pairs)

read by the pool leader (pools.remote) and the engine (collective-trip hooks).  Keys:
  die_on=MARK            a pool leader exits when a prompt contains MARK
  die_after=N            a pool leader exits after N generate / submit requests (with die_rank=R:
                         only on global rank R)
  die_on_data_ping=1     a pool leader exits during a data-plane ping
  hang_on=MARK, hang_s=S a request whose prompt contains MARK sleeps S seconds before generating
  ping_delay_n=N, ping_delay_s=S   the first N control-plane pings stall the receiver S seconds
  car_trip_decode=N, car_trip_prefill=N   force a one-shot all-reduce trip on step N (every rank)
  car_vote_decode=N, car_vote_rank=R      rank R raises its all-reduce flag during step N's vote
The reference has no fault injection; these hooks drive the failover tests.
"""
from __future__ import annotations

import os
from typing import Any, Dict

_cache: Dict[str, Dict[str, str]] = {}


def _parse(raw: str) -> Dict[str, str]:
    out = {}
    for part in raw.split(","):
        if "=" in part:
            k, v = part.split("=", 1)
            out[k.strip()] = v.strip()
    return out


def fault(key: str, default: Any = None, cast=str) -> Any:
    """Value of fault ``key`` from DLLM_FAULT (``default`` when unset)."""
    raw = os.environ.get("DLLM_FAULT", "")
    if not raw:
        return default
    spec = _cache.get(raw)
    if spec is None:
        spec = _cache[raw] = _parse(raw)
    v = spec.get(key)
    return default if v is None else cast(v)


def diag(name: str):
    """Diagnostics switch from ``DLLM_DIAG`` (comma-separated): ``sync`` (per-step host prep / wait
    log of the pipelined step loop), ``cpu`` (per-thread CPU share of the bench window),
    ``profile=PATH`` (cProfile of the bench's driver thread).  Returns the value for ``key=value``
    entries, True for bare names, None when absent."""
    raw = os.environ.get("DLLM_DIAG", "")
    for part in raw.split(","):
        k, _, v = part.strip().partition("=")
        if k == name:
            return v or True
    return None


def spec(**kw) -> str:
    """DLLM_FAULT value for keyword faults (tests): ``spec(die_after=1, die_rank=2)``."""
    return ",".join(f"{k}={v}" for k, v in kw.items())
