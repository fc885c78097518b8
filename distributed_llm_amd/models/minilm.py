"""MiniLM-L6 sentence encoder (all-MiniLM-L6-v2 architecture) on the HIP op library.

The reference embeds every query with sentence-transformers on the host CPU
(src/query_router_engine.py:181 and :571 — twice per query when hybrid + cache are on).
Here the encoder runs on the GPU in bf16: 6 BERT layers, H=384, 12 heads x 32, FFN 1536,
post-LN residual blocks (HIP LayerNorm+residual kernel), GELU (HIP), bidirectional attention,
masked mean-pool + L2 normalise (one HIP kernel).  Batched: one forward per batch of queries.
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
        self._memo_size = memo_size
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
        cfg = self.cfg
        toks = [self.tok.encode(t, max_len) for t in texts]
        B, S = len(toks), max(len(x) for x in toks)
        ids = torch.zeros((B, S), dtype=torch.int64)
        for i, x in enumerate(toks):
            ids[i, :len(x)] = torch.tensor(x)
        lens = torch.tensor([len(x) for x in toks], dtype=torch.int32)
        ids, lens_d = ids.to(self.device), lens.to(self.device)
        H, nh = cfg.hidden, cfg.heads
        x = F.embedding(ids, self.word) + self.pos[:S].unsqueeze(0) + self.type0
        x = ops.layer_norm(x.reshape(B * S, H).contiguous(), *self.emb_ln, cfg.eps)
        keymask = (torch.arange(S, device=self.device)[None, :] < lens_d[:, None])  # [B, S]
        attn_mask = keymask[:, None, None, :]
        for L in self.layers:
            qkv = F.linear(x, L["wqkv"], L["bqkv"]).view(B, S, 3, nh, H // nh).permute(2, 0, 3, 1, 4)
            a = F.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2], attn_mask=attn_mask)
            a = a.permute(0, 2, 1, 3).reshape(B * S, H)
            h = F.linear(a, L["wo"], L["bo"])
            x = ops.layer_norm(h, *L["ln1"], cfg.eps, residual=x.clone())  # post-LN: LN(attn + x)
            f = F.linear(ops.gelu(F.linear(x, L["w1"], L["b1"])), L["w2"], L["b2"])
            x = ops.layer_norm(f, *L["ln2"], cfg.eps, residual=x.clone())
        return ops.mean_pool_l2(x.view(B, S, H), lens_d)

    def encode(self, texts: List[str], max_len: int = 256) -> torch.Tensor:
        """[n, 384] f32 unit vectors on the device; memoised per text."""
        out: List[Optional[torch.Tensor]] = [None] * len(texts)
        todo: Dict[str, List[int]] = {}
        with self._lock:
            for i, t in enumerate(texts):
                v = self._memo.get(t)
                if v is None:
                    todo.setdefault(t, []).append(i)
                else:
                    self._memo.move_to_end(t)
                    out[i] = v
        if todo:
            keys = list(todo)
            embs = self._forward(keys, max_len)
            with self._lock:
                for k, e in zip(keys, embs):
                    for i in todo[k]:
                        out[i] = e
                    self._memo[k] = e
                while len(self._memo) > self._memo_size:
                    self._memo.popitem(last=False)
        return torch.stack(out) if out else torch.zeros((0, self.cfg.hidden), device=self.device)
