"""Engine-level GPU checks at the TRUE shapes of every BASELINE model family.

Each family runs as a 2-layer truncation at its real hidden size, intermediate size, head
count, KV-head count, head dim and vocabulary (models.configs), random-init bf16 weights:

  * HIP forward (prefill over a fresh prompt, then one decode token against the cached KV) vs
    a plain-PyTorch **fp32** reference of the same weights on the CPU (ops.reference, every
    weight upcast to f32, f32 KV caches);
  * hipGraph decode replay == eager decode, token for token, through the serving engine.

Families: llama-3.2-1b (d 64, G 4, V 128256, tied), llama-3-8b (d 128, G 4), llama-3-70b
(H 8192, I 28672, G 8), phi3-mini (d 96, G 1, MHA), mixtral-8x7b (8 experts top-2, I 14336),
tinyllama-1.1b (d 64, G 8).  The reference's own tiers are phi3-mini and llama3-8B
(/root/reference/src/devices/nano_api.py:15-16, orin_api.py:17-18).
"""
import copy

import pytest
import torch

from distributed_llm_amd import ops
from distributed_llm_amd.engine.llm_engine import LLMEngine
from distributed_llm_amd.engine.sampling import SamplingParams
from distributed_llm_amd.models.configs import get_model_config
from distributed_llm_amd.models.llama import AttnMeta

pytestmark = pytest.mark.gpu

FAMILIES = ["tinyllama-1.1b", "llama-3.2-1b", "llama-3-8b", "phi3-mini", "mixtral-8x7b", "llama-3-70b"]
PROMPT = ("user: explain how paged attention stores the key value cache in fixed size blocks, "
          "and why continuous batching needs it\nassistant:")


def _engine(name, **kw):
    cfg = get_model_config(name, n_layers=2)
    kw.setdefault("kv_cache_gb", 0.25)
    kw.setdefault("max_num_seqs", 8)
    kw.setdefault("max_model_len", 2048)
    return LLMEngine(cfg, device="cuda", **kw)


def _fp32_cpu_copy(m):
    """The same model on the CPU with every weight upcast to f32 (ops dispatch to ops.reference)."""
    mc = copy.copy(m)
    mc.device = torch.device("cpu")
    mc.dtype = torch.float32
    f = lambda t: t.detach().float().cpu()
    mc.embed = f(m.embed)
    mc.lm_head = mc.embed if m.lm_head is m.embed else f(m.lm_head)
    mc.final_norm = f(m.final_norm)
    mc.layers = [{k: f(v) for k, v in L.items()} for L in m.reference_layers()]
    mc.fused = False
    mc.moe_tg = False          # reference_layers() already restored the plain w13 layout
    mc.cos_sin = m.cos_sin.cpu()
    return mc


def _meta(ids_len, ctx, slots, table, G, dev):
    I = lambda x, dt=torch.int32: torch.tensor(x, dtype=dt, device=dev)
    ts, tt = ops.build_tiles([ids_len], G)
    return AttnMeta(I(slots), I([table]), I([0]), I([ids_len]), I([ctx]), I(ts), I(tt), I([ids_len - 1], torch.int64))


def _rel(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return float((a - b).norm() / b.norm().clamp(min=1e-6)), float(torch.nn.functional.cosine_similarity(a, b, dim=0))


@pytest.mark.parametrize("name", FAMILIES)
def test_true_shape_forward_matches_fp32_reference(name):
    eng = _engine(name, use_graphs=False)
    m = eng.model
    ids = eng.tok.encode(PROMPT)
    T = len(ids)
    sid = 4242
    table, _ = eng.bm.allocate(sid, ids + [0])
    G = m.nq // m.nkv
    dev = torch.device("cuda")
    # prefill (T tokens) then one decode token at position T
    meta_p = _meta(T, T, eng.bm.slots(sid, 0, T), table, G, dev)
    meta_d = _meta(1, T + 1, eng.bm.slots(sid, T, T + 1), table, G, dev)
    pos_p = torch.arange(T, dtype=torch.int32, device=dev)
    pos_d = torch.tensor([T], dtype=torch.int32, device=dev)
    ids_p = torch.tensor(ids, dtype=torch.int32, device=dev)
    ids_d = torch.tensor([ids[-1]], dtype=torch.int32, device=dev)
    hp = m.hidden_states(ids_p, pos_p, meta_p, eng.kv_caches)
    hd = m.hidden_states(ids_d, pos_d, meta_d, eng.kv_caches)
    lg = m.logits(hd).float().cpu()
    hp, hd = hp.float().cpu(), hd.float().cpu()

    mc = _fp32_cpu_copy(m)
    kv = [(torch.zeros(k.shape, dtype=torch.float32), torch.zeros(v.shape, dtype=torch.float32))
          for k, v in eng.kv_caches]
    C = lambda mt: AttnMeta(*(x.cpu() for x in (mt.slots, mt.block_tables, mt.qstart, mt.qlen, mt.ctx,
                                                 mt.tile_seq, mt.tile_tok0, mt.last_idx)))
    rp = mc.hidden_states(ids_p.cpu(), pos_p.cpu(), C(meta_p), kv)
    rd = mc.hidden_states(ids_d.cpu(), pos_d.cpu(), C(meta_d), kv)
    ref_logits = rd @ mc.lm_head.t()
    eng.bm.free(sid)
    for what, a, b in (("prefill", hp, rp), ("decode", hd, rd), ("logits", lg, ref_logits)):
        rel, cos = _rel(a, b)
        assert rel < 3e-2 and cos > 0.9995, f"{name} {what}: rel L2 {rel:.4f}, cosine {cos:.6f}"
    # greedy token agrees unless the reference's top-2 logits are within bf16 noise
    top2 = ref_logits[0].topk(2).values
    if float(top2[0] - top2[1]) > 0.05 * float(ref_logits[0].abs().max()):
        assert int(lg[0].argmax()) == int(ref_logits[0].argmax())


@pytest.mark.parametrize("name", FAMILIES)
def test_true_shape_graph_replay_matches_eager(name):
    prompts = [PROMPT, "user: hi", "user: " + "long context words " * 30]
    sp = SamplingParams(max_new_tokens=10)
    g = _engine(name, use_graphs=True)
    a = [o.token_ids for o in g.generate(prompts, sp)]
    del g
    torch.cuda.empty_cache()
    e = _engine(name, use_graphs=False)
    b = [o.token_ids for o in e.generate(prompts, sp)]
    assert a == b, name
    assert all(len(t) == 10 for t in a)
