"""MiniLM-L6 sentence encoder (all-MiniLM-L6-v2 architecture) on the HIP op library.

The reference embeds every query with sentence-transformers on the host CPU
(src/query_router_engine.py:181 and :571 — twice per query when hybrid + cache are on).
Here the encoder runs on the GPU in bf16 on our own kernels: 6 BERT layers, H=384, 12 heads x
32, FFN 1536, post-LN residual blocks.  Embedding sum + LayerNorm is one kernel; each projection
is one tgemm launch with its bias (and GELU, or the residual add) in the epilogue; attention is
the bidirectional MFMA kernel of csrc/kernels/encoder.hip; masked mean-pool + L2 normalise is one
kernel.  Batched: one forward per batch of queries.
Weights: HF ``model.safetensors`` of all-MiniLM-L6-v2 if provided, else random (seeded).
Tokenizer: BERT WordPiece via ``tokenizers`` when a vocab file is given, else a deterministic
hashing word tokenizer (vocab 30522).
"""
from __future__ import annotations

import hashlib
import os
import re
import threading
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from .. import ops

_WORD = re.compile(r"[a-z0-9]+|[^\sa-z0-9]")


@dataclass(frozen=True)
class MiniLMConfig:
    vocab: int = 30522
    hidden: int = 384
    layers: int = 6
    heads: int = 12
    intermediate: int = 1536
    max_position: int = 512
    eps: float = 1e-12


class _HashWordTokenizer:
    CLS, SEP, PAD = 101, 102, 0

    def __init__(self, vocab: int):
        self.vocab = vocab

    def encode(self, text: str, max_len: int) -> List[int]:
        ids = [self.CLS]
        for w in _WORD.findall(text.lower()):
            h = int.from_bytes(hashlib.blake2b(w.encode(), digest_size=4).digest(), "little")
            ids.append(1000 + h % (self.vocab - 1000))
        ids = ids[:max_len - 1] + [self.SEP]
        return ids


class _WordPiece:
    def __init__(self, vocab_file: str):
        from tokenizers import BertWordPieceTokenizer
        self.tok = BertWordPieceTokenizer(vocab_file, lowercase=True)

    def encode(self, text: str, max_len: int) -> List[int]:
        ids = self.tok.encode(text).ids
        return ids[:max_len - 1] + ids[-1:] if len(ids) > max_len else ids


class MiniLMEncoder:
    def __init__(self, cfg: MiniLMConfig = MiniLMConfig(), device="cuda", dtype=torch.bfloat16, seed: int = 1234,
                 vocab_file: Optional[str] = None, memo_size: int = 65536):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        H, I = cfg.hidden, cfg.intermediate
        rnd = lambda *s: (torch.randn(*s, generator=g) * 0.02).to(self.device, dtype)
        ones = lambda n: torch.ones(n, device=self.device, dtype=dtype)
        zeros = lambda n: torch.zeros(n, device=self.device, dtype=dtype)
        self.word = rnd(cfg.vocab, H)
        self.pos = rnd(cfg.max_position, H)
        self.type0 = rnd(H)
        self.emb_ln = (ones(H), zeros(H))
        self.layers = []
        for _ in range(cfg.layers):
            self.layers.append({
                "wqkv": rnd(3 * H, H), "bqkv": zeros(3 * H), "wo": rnd(H, H), "bo": zeros(H),
                "ln1": (ones(H), zeros(H)), "w1": rnd(I, H), "b1": zeros(I), "w2": rnd(H, I), "b2": zeros(H),
                "ln2": (ones(H), zeros(H))})
        vocab_file = vocab_file or os.environ.get("DLLM_MINILM_VOCAB")
        self.tok = _WordPiece(vocab_file) if vocab_file and os.path.exists(vocab_file) else _HashWordTokenizer(cfg.vocab)
        self._memo: "OrderedDict[str, torch.Tensor]" = OrderedDict()
        # per-text memo of embeddings (DLLM_ENCODER_MEMO=0 disables it: every query is encoded)
        self._memo_size = memo_size if os.environ.get("DLLM_ENCODER_MEMO", "1") != "0" else 0
        self.memo_hits = self.memo_misses = self.encoded_texts = self.batch_hits = 0
        # embeddings of the current routing batch (prefetch): reused by the batch's own lookups
        # (semantic router + semantic cache) even with the memo off, replaced by the next batch
        self._scope: Dict[str, torch.Tensor] = {}
        self._lock = threading.Lock()

    def load_safetensors(self, path: str) -> None:
        from safetensors.torch import load_file
        t = load_file(path)
        p = "" if "embeddings.word_embeddings.weight" in t else "bert."
        put = lambda x: x.to(self.device, self.dtype).contiguous()
        self.word = put(t[p + "embeddings.word_embeddings.weight"])
        self.pos = put(t[p + "embeddings.position_embeddings.weight"])
        self.type0 = put(t[p + "embeddings.token_type_embeddings.weight"][0])
        self.emb_ln = (put(t[p + "embeddings.LayerNorm.weight"]), put(t[p + "embeddings.LayerNorm.bias"]))
        for i, L in enumerate(self.layers):
            q = f"{p}encoder.layer.{i}."
            a = q + "attention.self."
            L["wqkv"] = put(torch.cat([t[a + n + ".weight"] for n in ("query", "key", "value")]))
            L["bqkv"] = put(torch.cat([t[a + n + ".bias"] for n in ("query", "key", "value")]))
            L["wo"] = put(t[q + "attention.output.dense.weight"])
            L["bo"] = put(t[q + "attention.output.dense.bias"])
            L["ln1"] = (put(t[q + "attention.output.LayerNorm.weight"]), put(t[q + "attention.output.LayerNorm.bias"]))
            L["w1"] = put(t[q + "intermediate.dense.weight"])
            L["b1"] = put(t[q + "intermediate.dense.bias"])
            L["w2"] = put(t[q + "output.dense.weight"])
            L["b2"] = put(t[q + "output.dense.bias"])
            L["ln2"] = (put(t[q + "output.LayerNorm.weight"]), put(t[q + "output.LayerNorm.bias"]))
        with self._lock:
            self._memo.clear()

    @torch.no_grad()
    def _forward(self, texts: List[str], max_len: int) -> torch.Tensor:
        """One padded batch through the HIP encoder: fused embedding+LN, per layer 4 tgemm launches
        (QKV + bias, Wo + bias + residual, W1 + bias + GELU, W2 + bias + residual), the encoder
        attention kernel and 2 LayerNorms; masked mean-pool + L2 (csrc/kernels/encoder.hip,
        tgemm.hip, norm.hip, cosine.hip).  CPU tensors run the same graph on ops.reference."""
        cfg = self.cfg
        toks = [self.tok.encode(t, max_len) for t in texts]
        B, S = len(toks), max(len(x) for x in toks)
        ids = torch.zeros((B, S), dtype=torch.int32)
        for i, x in enumerate(toks):
            ids[i, :len(x)] = torch.tensor(x, dtype=torch.int32)
        lens = torch.tensor([len(x) for x in toks], dtype=torch.int32)
        ids, lens_d = ids.to(self.device), lens.to(self.device)
        H, nh = cfg.hidden, cfg.heads
        x = ops.embed_ln(ids, self.word, self.pos, self.type0, *self.emb_ln, S, cfg.eps)
        for L in self.layers:
            qkv = ops.gemm.linear_bias(x, L["wqkv"], L["bqkv"])
            a = ops.encoder_attention(qkv, lens_d, B, S, nh, H // nh)
            x = ops.layer_norm(ops.gemm.linear_bias_residual(a, L["wo"], L["bo"], x), *L["ln1"], cfg.eps)
            f = ops.gemm.linear_bias(x, L["w1"], L["b1"], gelu=True)
            x = ops.layer_norm(ops.gemm.linear_bias_residual(f, L["w2"], L["b2"], x), *L["ln2"], cfg.eps)
        return ops.mean_pool_l2(x.view(B, S, H), lens_d)

    @torch.no_grad()
    def reference_forward(self, texts: List[str], max_len: int = 256) -> torch.Tensor:
        """fp32 PyTorch forward of the same weights (numerics oracle for the HIP path)."""
        cfg = self.cfg
        toks = [self.tok.encode(t, max_len) for t in texts]
        B, S = len(toks), max(len(x) for x in toks)
        ids = torch.zeros((B, S), dtype=torch.int64)
        for i, x in enumerate(toks):
            ids[i, :len(x)] = torch.tensor(x)
        lens = torch.tensor([len(x) for x in toks])
        f = lambda t: t.detach().float().cpu()
        H, nh = cfg.hidden, cfg.heads
        x = f(self.word)[ids] + f(self.pos)[:S][None] + f(self.type0)
        x = F.layer_norm(x, (H,), f(self.emb_ln[0]), f(self.emb_ln[1]), cfg.eps)
        keymask = (torch.arange(S)[None, :] < lens[:, None])[:, None, None, :]
        for L in self.layers:
            qkv = F.linear(x, f(L["wqkv"]), f(L["bqkv"])).view(B, S, 3, nh, H // nh).permute(2, 0, 3, 1, 4)
            a = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2], attn_mask=keymask)
            a = a.permute(0, 2, 1, 3).reshape(B, S, H)
            x = F.layer_norm(x + F.linear(a, f(L["wo"]), f(L["bo"])), (H,), f(L["ln1"][0]), f(L["ln1"][1]), cfg.eps)
            h = F.linear(F.gelu(F.linear(x, f(L["w1"]), f(L["b1"]))), f(L["w2"]), f(L["b2"]))
            x = F.layer_norm(x + h, (H,), f(L["ln2"][0]), f(L["ln2"][1]), cfg.eps)
        m = (torch.arange(S)[None, :] < lens[:, None]).float()[..., None]
        return F.normalize((x * m).sum(1) / m.sum(1).clamp(min=1.0), dim=-1)

    def prefetch(self, texts: List[str], max_len: int = 256) -> None:
        """One batched forward for a routing batch's unique texts (memo hits excluded); the
        results serve this batch's per-query lookups."""
        uniq = list(dict.fromkeys(texts))
        with self._lock:
            todo = [t for t in uniq if not (self._memo_size and t in self._memo)]
        scope: Dict[str, torch.Tensor] = {}
        if todo:
            embs = self._forward(todo, max_len)
            scope = dict(zip(todo, embs))
        with self._lock:
            self.encoded_texts += len(todo)
            if self._memo_size:
                for k, e in scope.items():
                    self._memo[k] = e
                while len(self._memo) > self._memo_size:
                    self._memo.popitem(last=False)
            self._scope = scope

    def memo_stats(self) -> Dict[str, float]:
        n = self.memo_hits + self.memo_misses + self.batch_hits
        return {"memo_enabled": bool(self._memo_size), "lookups": n, "hits": self.memo_hits,
                "hit_rate": round(self.memo_hits / n, 4) if n else 0.0, "encoded_texts": self.encoded_texts,
                "batch_hits": self.batch_hits}

    def encode(self, texts: List[str], max_len: int = 256) -> torch.Tensor:
        """[n, 384] f32 unit vectors on the device; memoised per text."""
        out = self.encode_rows(texts, max_len)
        return torch.stack(out) if out else torch.zeros((0, self.cfg.hidden), device=self.device)

    def encode_rows(self, texts: List[str], max_len: int = 256) -> List[torch.Tensor]:
        """``encode`` as one [384] row view per text, with no stacking launch: the rows belong to
        forward outputs that are never written again (the routing cache keeps references)."""
        out: List[Optional[torch.Tensor]] = [None] * len(texts)
        todo: Dict[str, List[int]] = {}
        with self._lock:
            scoped = 0
            for i, t in enumerate(texts):
                v = self._memo.get(t) if self._memo_size else None
                if v is not None:
                    self._memo.move_to_end(t)
                    out[i] = v
                elif t in self._scope:
                    out[i] = self._scope[t]
                    scoped += 1
                else:
                    todo.setdefault(t, []).append(i)
            missed = sum(len(v) for v in todo.values())
            self.batch_hits += scoped
            self.memo_hits += len(texts) - missed - scoped
            self.memo_misses += missed
            self.encoded_texts += len(todo)
        if todo:
            keys = list(todo)
            embs = self._forward(keys, max_len)
            with self._lock:
                for k, e in zip(keys, embs):
                    for i in todo[k]:
                        out[i] = e
                    if self._memo_size:
                        self._memo[k] = e
                while len(self._memo) > self._memo_size:
                    self._memo.popitem(last=False)
        return out
