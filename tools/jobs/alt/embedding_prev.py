"""Text embedders for the semantic store.

`HashingEmbedder` (default): signed feature hashing of lower-cased word unigrams
and bigrams plus character trigrams into D=1024 dims, L2-normalised. It is
deterministic, needs no weights, and makes cosine similarity track lexical
overlap — a strict generalisation of the reference's case-insensitive
substring search (pilott/memory/enhanced_memory.py:110), which it replaces.

`EngineEmbedder`: mean-pooled final hidden states of the local Llama engine's model,
projected to D by a fixed random orthogonal map (meaningful with real weights). By
default (`pool="engine"`) the texts go through the serving engine itself as embedding
requests — same kernels, same continuous batch as the agents' calls.
"""
from __future__ import annotations

import re
import zlib
from typing import List, Sequence

import numpy as np

_TOK = re.compile(r"[a-z0-9]+")


def _h(s: str) -> int:
    return zlib.crc32(s.encode("utf-8"))


class HashingEmbedder:
    def __init__(self, dim: int = 1024):
        self.dim = dim

    def features(self, text: str):
        t = text.lower()
        words = _TOK.findall(t)
        feats = [("w", w) for w in words]
        feats += [("b", f"{a} {b}") for a, b in zip(words, words[1:])]
        squeezed = " ".join(words)
        feats += [("c", squeezed[i:i + 3]) for i in range(max(0, len(squeezed) - 2))]
        return feats

    def embed(self, texts: Sequence[str]) -> np.ndarray:
        out = np.zeros((len(texts), self.dim), dtype=np.float32)
        wts = {"w": 1.0, "b": 0.7, "c": 0.35}
        for r, text in enumerate(texts):
            row = out[r]
            for kind, f in self.features(text):
                h = _h(kind + ":" + f)
                row[h % self.dim] += wts[kind] * (1.0 if (h >> 31) & 1 else -1.0)
            n = np.linalg.norm(row)
            if n > 0:
                row /= n
        return out

    def __call__(self, texts: Sequence[str]) -> np.ndarray:
        return self.embed(texts)


class EngineEmbedder:
    """Embeddings from the serving model itself: final-norm hidden states
    mean-pooled over the text's tokens (pooling="last": the last token's state, which lets
    the engine reuse cached prefixes), projected to `dim` by a fixed orthonormal matrix and
    L2-normalised; texts truncated to `max_tokens`.

    pool="engine" (default): embedding requests through `LLMEngine.embed` — prefilled by
    the engine's kernels inside its continuous batch, pooled in the step graph.
    pool="hidden": a separate dense PyTorch forward (LlamaModel.hidden_states), the
    reference the engine path is tested against. pool="tokens": the (much cheaper) mean
    of the input token embeddings."""

    def __init__(self, engine, dim: int = 1024, seed: int = 0, pool: str = "engine", batch_size: int = 16,
                 max_tokens: int = 512, pooling: str = "mean"):
        import torch

        self.engine = engine
        self.dim = dim
        d = engine.model_cfg.hidden_size
        g = torch.Generator().manual_seed(seed)
        if d >= dim:  # [d, dim] with orthonormal columns
            q, _ = torch.linalg.qr(torch.randn(d, dim, generator=g))
        else:  # a model narrower than the index (test shapes): orthonormal rows
            q = torch.linalg.qr(torch.randn(dim, d, generator=g))[0].T
        self.proj = q.contiguous().to(engine.device, torch.float32)
        self.pool = pool if (pool == "engine" or getattr(engine.model.tp, "size", 1) == 1) else "tokens"
        self.batch_size = batch_size
        self.max_tokens = max_tokens
        if pooling not in ("mean", "last"):
            raise ValueError(f"pooling must be 'mean' or 'last', not {pooling!r}")
        # "last": the last token's state — embedding requests then reuse the engine's prefix
        # cache (texts that share a prefix, like an agent's successive lookups, share its work)
        self.pooling = pooling

    def embed(self, texts: Sequence[str]) -> np.ndarray:
        import torch
        import torch.nn.functional as F

        m = self.engine.model
        rows: List[np.ndarray] = []
        if self.pool == "engine":
            ids = [self.engine.tok.encode(t)[: self.max_tokens] or [0] for t in texts]
            if not ids:
                return np.zeros((0, self.dim), np.float32)
            h = torch.from_numpy(self.engine.embed(ids, pooling=self.pooling)).to(self.proj.device)
            return F.normalize(h @ self.proj, dim=1).cpu().numpy()
        with torch.inference_mode():
            if self.pool == "hidden":
                for i in range(0, len(texts), self.batch_size):
                    ids = [self.engine.tok.encode(t)[: self.max_tokens] or [0] for t in texts[i:i + self.batch_size]]
                    v = F.normalize(m.hidden_states(ids, pooling=self.pooling) @ self.proj, dim=1)
                    rows.extend(v.cpu().numpy())
            else:
                for t in texts:
                    ids = torch.tensor(self.engine.tok.encode(t)[: self.max_tokens] or [0], device=self.engine.device)
                    h = F.embedding(ids, m.embed).float().mean(0)
                    rows.append(F.normalize(h @ self.proj, dim=0).cpu().numpy())
        return np.stack(rows) if rows else np.zeros((0, self.dim), np.float32)

    def __call__(self, texts):
        return self.embed(texts)
