"""Is the engine's greedy decode deterministic?  (round 5: one run of
tests/test_models_gpu.py::test_true_shape_graph_replay_matches_eager[mixtral-8x7b] disagreed at one
token, the rerun passed.)  Runs the 2-layer true-shape engine several times with and without
graphs on the test's prompts and prints which runs agree."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from distributed_llm_amd.engine.llm_engine import LLMEngine  # noqa: E402
from distributed_llm_amd.engine.sampling import SamplingParams  # noqa: E402
from distributed_llm_amd.models.configs import get_model_config  # noqa: E402

PROMPT = ("user: explain how paged attention stores the key value cache in fixed size blocks, "
          "and why continuous batching needs it\nassistant:")


def run(name, graphs, n):
    prompts = [PROMPT, "user: hi", "user: " + "long context words " * 30]
    sp = SamplingParams(max_new_tokens=24)
    outs = []
    for _ in range(n):
        e = LLMEngine(get_model_config(name, n_layers=2), device="cuda", kv_cache_gb=0.25, max_num_seqs=8,
                      max_model_len=2048, use_graphs=graphs)
        outs.append([o.token_ids for o in e.generate(prompts, sp)])
        del e
        torch.cuda.empty_cache()
    return outs


def op_repeats(n=20):
    """Bitwise run-to-run check of the MoE ops on fixed inputs (Mixtral-like, narrowed)."""
    from distributed_llm_amd import ops
    torch.manual_seed(0)
    dev = "cuda"
    res = {}
    for T in (3, 96, 700):
        H, I, E, k = 1024, 1024, 8, 2
        x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
        lg = torch.randn(T, E, device=dev)
        ids, w = ops.moe_gate(lg, k)
        w13 = torch.randn(E, 2 * I, H, device=dev, dtype=torch.bfloat16) * 0.03
        w2 = torch.randn(E, H, I, device=dev, dtype=torch.bfloat16) * 0.03
        y0 = ops.moe_ffn_tg(x, ids, w, w13, w2)
        g0 = ops.moe_gate(lg, k)
        bad_y = sum(int(not torch.equal(ops.moe_ffn_tg(x, ids, w, w13, w2), y0)) for _ in range(n))
        bad_g = sum(int(not all(torch.equal(a, b) for a, b in zip(ops.moe_gate(lg, k), g0))) for _ in range(n))
        res[f"T{T}"] = {"moe_ffn_tg_mismatch": bad_y, "moe_gate_mismatch": bad_g}
    print(json.dumps({"op_repeats": res}), flush=True)


def main():
    op_repeats()
    for name in sys.argv[1:] or ["mixtral-8x7b", "llama-3-8b"]:
        g, e = run(name, True, 3), run(name, False, 3)
        base = e[0]
        diff = lambda a: [next((i for i, (x, y) in enumerate(zip(p, q)) if x != y), None) for p, q in zip(a, base)]
        print(json.dumps({"model": name, "graph_vs_eager0_first_diff": [diff(a) for a in g],
                          "eager_vs_eager0_first_diff": [diff(a) for a in e]}), flush=True)


if __name__ == "__main__":
    main()
