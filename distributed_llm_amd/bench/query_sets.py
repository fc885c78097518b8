"""Benchmark query sets (reference ``src/tests/query_sets.py``; data in ``data/query_sets.json``)
and the harness's normaliser (reference ``src/tests/routing_chatbot_tester.py:75-109``)."""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

from ..config import QUERY_SET_PATH


@dataclass
class QueryItem:
    text: str
    expected_device: Optional[str] = None


def _load() -> Dict[str, List[Dict[str, str]]]:
    with open(QUERY_SET_PATH, "r", encoding="utf-8") as f:
        raw = json.load(f)
    return {k: [{"query": q, "expected_device": e} for q, e in v] for k, v in raw.items() if not k.startswith("_")}


query_sets: Dict[str, List[Dict[str, str]]] = _load()


def normalize_query_set(raw_items: Any) -> List[QueryItem]:
    """Accept list[str] or list[dict(query|text, expected_device|label)]."""
    if not isinstance(raw_items, list):
        raise ValueError("query set must be a list")
    out: List[QueryItem] = []
    for x in raw_items:
        if isinstance(x, str):
            if x.strip():
                out.append(QueryItem(x.strip()))
        elif isinstance(x, dict):
            q = (x.get("query") or x.get("text") or "").strip()
            if not q:
                continue
            exp = x.get("expected_device") or x.get("label")
            exp = exp.lower().strip() if isinstance(exp, str) else None
            out.append(QueryItem(q, exp if exp in ("nano", "orin") else None))
    if not out:
        raise ValueError("Query set is empty after normalization")
    return out
