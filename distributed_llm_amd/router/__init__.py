"""Query Routing Engine: strategies, predictive cache, QueryRouter (reference L4)."""
from .cache import CacheEntry, CacheLookupResult, QueryCache, RoutingRecord, EmbeddingIndex
from .embedder import Embedder, HashEmbedder, get_embedder
from .query_router import QueryRouter
from .strategies import (STRATEGIES, BaseRouter, HeuristicRouter, HybridRouter,
                         PerformanceAwareRouter, RoutingDecision, SemanticRouter, TokenBasedRouter)
from .tokens import TokenCounter

__all__ = [
    "CacheEntry", "CacheLookupResult", "QueryCache", "RoutingRecord", "EmbeddingIndex",
    "Embedder", "HashEmbedder", "get_embedder", "QueryRouter", "STRATEGIES", "BaseRouter",
    "HeuristicRouter", "HybridRouter", "PerformanceAwareRouter", "RoutingDecision",
    "SemanticRouter", "TokenBasedRouter", "TokenCounter",
]
