"""distributed_llm_amd — MI355X-native heterogeneous query-routing inference engine.

Layers (new mapping):
  server/    HTTP API (/chat, /history) + CLI REPL            (reference L6/L7)
  orchestrator  Router.route_query contract                    (reference L5)
  router/    five strategies, predictive cache, QueryRouter    (reference L4)
  pools/     pool clients, pool-worker HTTP shim, supervisor   (reference L2/L3)
  engine/    paged-KV LLM engine, scheduler, hipGraph runner   (replaces Ollama, L1)
  models/    Llama / Phi-3 / Mixtral / MiniLM definitions
  ops/       HIP/CDNA4 kernels (csrc/kernels) + torch references
  parallel/  RCCL communicators, tensor-parallel layers, P2P failover/probes
  bench/     benchmark harnesses (reference CSV schemas), power sampling, query sets
"""
__version__ = "0.1.0"
