"""Llama-3 decoder (8B / 70B / tiny test shapes) for the on-node inference engine.

The forward is written for a ragged token batch (prefill chunks + decode tokens
+ grammar jump-forward runs in one pass, see runtime/scheduler.cpp) over a paged
KV cache, and is hipGraph-capturable: every device-side shape is fixed by the
token bucket, all per-step metadata lives in one device buffer that the host
refreshes with a single H2D copy.

Per layer on the packed-weight paths (every step of a Llama-3 model that fits two weight
copies; decode / mid / prefill by step size, see forward()):
  QKV projection (RMSNorm folded into the weights, RoPE + paged KV write in the epilogue)
  -> paged GQA attention (csrc/ops/attention.hip, MFMA) -> O projection (+ residual, next
  norm's row statistics) [TP: all-reduce] -> gate_up (norm folded, SwiGLU epilogue)
  -> down (+ residual, statistics) [TP: all-reduce]
all on hand-written gfx950 kernels (gemm_decode / gemm_stream / gemm_mid / gemm_prefill .hip).
The unpacked fallback (models too large for a second weight copy, e.g. 70B at TP=1) runs
rmsnorm -> library GEMM -> rope_cache -> attention -> GEMM -> add-norm -> GEMM -> SwiGLU -> GEMM.

Tensor parallelism: QKV and gate_up are column-parallel,
O and down are row-parallel followed by an all-reduce over RCCL/xGMI, the
embedding and LM head are vocab-parallel; sampling picks the global winner from
per-shard Gumbel keys (csrc/ops/sampling.hip via engine/engine.py), so TP=8 emits
exactly the TP=1 token.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from pilottai_amd import ops
from pilottai_amd.ops import reference as ref
from pilottai_amd.parallel.comm import TPGroup


@dataclass
class LlamaConfig:
    name: str = "llama-3-8b"
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    rms_eps: float = 1e-5
    max_position: int = 8192
    tie_embeddings: bool = False
    init_std: float = 0.02

    @property
    def gqa_group(self) -> int:
        return self.num_heads // self.num_kv_heads

    def num_params(self) -> int:
        d, f, v = self.hidden_size, self.intermediate_size, self.vocab_size
        qkv = d * (self.num_heads + 2 * self.num_kv_heads) * self.head_dim
        per_layer = qkv + self.num_heads * self.head_dim * d + 3 * d * f + 2 * d
        return self.num_layers * per_layer + v * d * (1 if self.tie_embeddings else 2) + d


PRESETS: Dict[str, LlamaConfig] = {
    "llama-3-8b": LlamaConfig(),
    "llama-3-70b": LlamaConfig(name="llama-3-70b", hidden_size=8192, intermediate_size=28672,
                               num_layers=80, num_heads=64, num_kv_heads=8),
    "llama-3.1-8b": LlamaConfig(name="llama-3.1-8b", max_position=131072,
                                rope_scaling={"factor": 8.0, "low_freq_factor": 1.0,
                                              "high_freq_factor": 4.0,
                                              "original_max_position_embeddings": 8192}),
    # test shapes: real head_dim / GQA layout, few layers, Llama-3 vocabulary
    "tiny": LlamaConfig(name="tiny", hidden_size=512, intermediate_size=1024, num_layers=2,
                        num_heads=4, num_kv_heads=1, max_position=4096),
    "tiny-gqa4": LlamaConfig(name="tiny-gqa4", hidden_size=1024, intermediate_size=2048,
                             num_layers=2, num_heads=8, num_kv_heads=2, max_position=4096),
    # 8 KV heads like Llama-3-8B/70B: shardable at TP = 2, 4 and 8 (TP tests)
    "tiny-kv8": LlamaConfig(name="tiny-kv8", hidden_size=1024, intermediate_size=2048, num_layers=2,
                            num_heads=16, num_kv_heads=8, max_position=4096),
    # the exact Llama-3-8B layer (4096 / 14336 / 32:8 heads / full vocabulary), 2 layers deep:
    # production shapes through every forward path at test cost
    "llama-3-8b-2l": LlamaConfig(name="llama-3-8b-2l", num_layers=2, max_position=4096),
    # the exact Llama-3-70B layer, 1 / 2 layers deep (per-layer launch counts of the TP step graph:
    # tools/graph_nodes.py)
    "llama-3-70b-1l": LlamaConfig(name="llama-3-70b-1l", hidden_size=8192, intermediate_size=28672,
                                  num_layers=1, num_heads=64, num_kv_heads=8, max_position=4096),
    "llama-3-70b-2l": LlamaConfig(name="llama-3-70b-2l", hidden_size=8192, intermediate_size=28672,
                                  num_layers=2, num_heads=64, num_kv_heads=8, max_position=4096),
}


def get_config(name_or_cfg) -> LlamaConfig:
    if isinstance(name_or_cfg, LlamaConfig):
        return name_or_cfg
    key = str(name_or_cfg).lower()
    if key not in PRESETS:
        raise ValueError(f"unknown model {name_or_cfg!r}; known: {sorted(PRESETS)}")
    return PRESETS[key]


@dataclass
class StepMeta:
    """Device views of one step's metadata (layout from the native scheduler)."""
    input_ids: torch.Tensor
    positions: torch.Tensor
    slots: torch.Tensor
    q_start: torch.Tensor
    q_len: torch.Tensor
    ctx_len: torch.Tensor
    block_table: torch.Tensor
    items: torch.Tensor
    n_items: torch.Tensor
    att_counters: torch.Tensor  # persistent zeroed workspace (partition tickets), not step data
    logit_rows: torch.Tensor
    num_seqs: int = 0  # host-side count, used only by the CPU reference path
    part_size: Optional[torch.Tensor] = None  # device int[1]: decode partition size of the step


class KVCache:
    """Per-layer paged pools (bf16): K [NB, KV, 128/8, 16, 8] fragment-major,
    V^T [NB, KV, 128, 16] (layouts: csrc/ops/rope_cache.hip)."""

    def __init__(self, num_layers: int, num_blocks: int, kv_heads: int, device, dtype=torch.bfloat16,
                 block_size: int = 16):
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.k = torch.zeros(num_layers, num_blocks, kv_heads, 16, block_size, 8, dtype=dtype, device=device)
        self.v = torch.zeros(num_layers, num_blocks, kv_heads, 128, block_size, dtype=dtype, device=device)

    @staticmethod
    def bytes_per_block(num_layers: int, kv_heads: int, block_size: int = 16) -> int:
        return 2 * num_layers * kv_heads * block_size * 128 * 2


DENSE_KINDS = ("wqkv", "wo", "w13", "w2")


class LlamaModel:
    # decode steps of at most this many tokens run the fused packed-weight path
    # (csrc/ops/gemm_decode.hip; tools/decode_gemm_bench.py, profiles/r1_decode_gemm.md)
    DECODE_FUSED_MAX_T = 16
    # steps of up to this many tokens (above DECODE_FUSED_MAX_T) run the LDS-DMA tiled projections
    # (csrc/ops/gemm_mid.hip) with every norm / SwiGLU / residual / RoPE + KV write fused
    MID_MAX_T = 256
    # steps above MID_MAX_T and up to this many tokens run the same fused packed-weight layer
    # with the prefill kernels (csrc/ops/gemm_prefill.hip) for the projections PF_CFG assigns
    # to them; no library GEMM and no separate norm / SwiGLU / RoPE launch.
    # EngineConfig.prefill_max_t / bench.py --prefill-max-t move the boundary (0 = off:
    # library GEMMs + elementwise kernels above MID_MAX_T).
    PREFILL_MAX_T = 1 << 30
    # projections whose PF_CFG prefill-kernel rows also apply to steps of <= MID_MAX_T tokens
    # (empty: the mid kernel takes every such step). In isolation the 256 x 128 prefill tiles
    # beat the mid kernel for every projection from 96-160 rows even with cold weights
    # (profiles/r3_midrange_cold_sweep.jsonl), but in the engine only gate_up keeps the gain
    # (144-256-token steps 0.1-0.2 ms faster in two alternating runs); qkv, o and down lose there
    # for a reason not isolated yet (their engine-exact epilogues cost the prefill kernels only
    # ~3 us, profiles/r3_epilogue_cost.jsonl) (profiles/r3_midrange_engine_ab.jsonl; tools/midrange_ab.py, one engine per choice, alternating:
    # profiles/r3_midrange_inengine_ab.jsonl — 160 / 192 / 256-token steps 6.20 / 6.35 / 6.73 ms
    # with the mid kernel, 5.96 / 6.11 / 6.59 with gate_up here, 6.72 / 6.89 / 7.22 with all four)
    PF_MIDRANGE = frozenset({"gate_up"})
    # steps of at most this many tokens (above DECODE_FUSED_MAX_T) run the QKV projection on the
    # packed decode kernel (all rows per workgroup, norm from x, RoPE + KV write; csrc/ops/
    # gemm_decode.hip handles M <= 64) instead of the mid kernel; 0 = off
    DEC_QKV_MAX_T = 0
    # waves per attention workgroup on decode-sized steps (T <= DECODE_FUSED_MAX_T): 8 splits
    # each item's chain of 32-key tiles over twice the waves (csrc/ops/attention.hip NW = 8), and
    # the scheduler then skips the flash-decoding split for such steps with few rows; 8-worker
    # bench 14.17 / 14.24 -> 14.41 / 14.47 tasks/s, 8-token steps 3.28 -> 3.19-3.20 ms
    # (profiles/r3_attention_8wave.jsonl)
    ATT_DECODE_WAVES = int(os.environ.get("PILOTTAI_ATT_DECODE_WAVES", "8"))
    # waves per attention workgroup on the mid path (DECODE_FUSED_MAX_T < T <= MID_MAX_T)
    ATT_MID_WAVES = int(os.environ.get("PILOTTAI_ATT_MID_WAVES", "4"))
    # per projection: (largest M, path, config); the first row whose M covers the step is used,
    # for every step on the fused packed-weight path (T > DECODE_FUSED_MAX_T).
    # "pf": prefill kernel — bn = tile width (256 / 128), variant = kernel family (3: the
    # ping-pong kernels of gemm_pingpong.h, 1: the read-ahead 256 x 256 / 3-stage 256 x 128
    # kernels), full / splits = the decomposition (-1 / 0: the kernel's plan); "mid": mid
    # kernel (fm, fn, splits as MID_CFG). Rows from tools/prefill_gemm_bench.py on MI355X
    # (profiles/r3_pingpong_gemm_bench_n128.jsonl: fastest fused kernel per shape and M above
    # 256 rows; profiles/r3_midrange_pf_vs_mid.jsonl: from 192 rows the 256 x 128 prefill tiles
    # beat the mid kernel's 128-256-row tiles, e.g. qkv 50.1 -> 27.5 us and o 40.9 -> 25.8 at
    # 256 rows, because the mid tiles' x panel leaves LDS room for one 64-k chunk in flight;
    # crossovers from profiles/r3_midrange_fused_sweep.jsonl: qkv above 80 rows, the others above 128).
    # qkv above 1,280 rows: 256 x 192 tiles (bn 192, N % 192 == 0, else 256) where their whole
    # rounds beat the 256 x 256 tiles' rounds + split tail: 1,281-2,048 rows (one round of 192-256
    # tiles instead of 144-192 wide ones) and from 3,841 (profiles/r5_qkv_192_tiles.jsonl: RoPE +
    # KV-write epilogue 71.9 / 77.1 / 84.7 / 164.3 us at 1,536 / 1,792 / 2,048 / 4,096 rows vs
    # 83.9 / 87.2 / 94.2 / 181.7 on 256 x 256 tiles; plain 2,048 rows 76.2 us vs hipBLASLt 80.1).
    # Round 5: the 256 x 128 ping-pong family (variant 3) replaced the 3-stage 256 x 128 kernel
    # (variant 1) in every row: 10-25 % faster in isolation at 144-1,280 rows for every projection
    # (profiles/r5_pf_family_sweep.jsonl, r5_midrange_isolated_sweep.jsonl; e.g. o at 512 rows
    # 32.6 vs 41.8 us, down at 384 rows 64.2 vs 76.2), and in the engine (alternating on one box,
    # profiles/r5_pf_family_inengine_ab.jsonl): headline bench 43.51 vs 42.89 tasks/s (3 reps),
    # 256- / 192-row steps 7.94 / 7.08 vs 8.05 / 7.17 ms; qkv of 129-256-row steps stays on the
    # mid kernel (on the prefill kernel there: 8.34 vs 7.94 ms at 256 rows)
    PF_CFG = {
        "qkv": [(80, "mid", {}), (1280, "pf", {"bn": 128, "variant": 3}),
                (2048, "pf", {"bn": 192, "variant": 3}), (3840, "pf", {"bn": 256, "variant": 3}),
                (1 << 30, "pf", {"bn": 192, "variant": 3})],
        "o": [(128, "mid", {}), (1 << 30, "pf", {"bn": 128, "variant": 3})],
        "gate_up": [(128, "mid", {}), (256, "pf", {"bn": 128, "variant": 3}),
                    (1 << 30, "pf", {"bn": 256, "variant": 3})],
        "down": [(128, "mid", {}), (512, "pf", {"bn": 128, "variant": 3}),
                 (1 << 30, "pf", {"bn": 256, "variant": 3})],
    }
    # per projection: (largest M, shape) rows for the weight-streaming kernel
    # (csrc/ops/gemm_stream.hip; shape = (rg, tpw, wt, wk, S, D): row groups, 16-column tiles
    # per wave, waves along N, waves along K, K-split, ring depth; the rows per group follow
    # from the step, _stream_plan); the first row whose M covers a mid-size step
    # (DECODE_FUSED_MAX_T < T <= MID_MAX_T) replaces PF_CFG / MID_CFG there.
    # Rows only where tools/stream_gemm_bench.py (graph-replayed, cold weights, engine
    # epilogues) measured it ahead of the round-3 choice (profiles/r4_stream_gemm_*.jsonl).
    # (profiles/r4_stream_gemm_sweep_final.jsonl, interleaved, cold weights, us stream vs round 3:
    #  o 32 / 64 / 128 rows: 13.4 / 14.6 / 18.9 vs 15.0 / 16.4 / 20.6 (256: 23.1 vs 22.3, not taken);
    #  down 32 / 64 / 128 / 256: 27.1 / 29.8 / 35.7 / 49.6 vs 29.0 / 34.0 / 46.3 / 62.5;
    #  qkv 32: 15.1 vs 16.0 (64 / 128 tie, 256 slower); gate_up: ties at 32, slower above)
    STREAM_CFG: Dict[str, list] = {
        "qkv": [(32, (1, 1, 4, 1, 2, 4))],
        "o": [(64, (1, 1, 4, 1, 4, 4)), (128, (1, 1, 4, 1, 4, 2))],
        "down": [(32, (1, 1, 4, 1, 4, 4)), (128, (1, 2, 4, 1, 8, 2)), (256, (2, 2, 8, 1, 7, 2))],
    }
    # LM head of steps with more than 32 logit rows (<= 32: the packed decode kernel):
    # (largest rows, shape as STREAM_CFG) on the weight-streaming kernel; empty = hipBLASLt
    # the (N, K) each projection's STREAM_CFG rows were measured on (Llama-3-8B at TP = 1); other
    # shapes (TP shards, other models) keep the round-3 choice. {} = rows apply to any shape.
    STREAM_NK: Dict[str, tuple] = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
                                   "down": (4096, 14336), "lm_head": (128256, 4096)}
    # (profiles/r4_stream_lm_head_sweep.jsonl: 24 / 48 / 64 / 128 rows 166 / 172 / 175 / 197 us
    # vs 176 (packed decode kernel) / 210 / 210 / 235 (hipBLASLt); 17-32 rows included)
    LM_HEAD_STREAM: list = [(32, (1, 3, 4, 1, 1, 2)), (64, (1, 4, 4, 1, 1, 2)), (128, (1, 2, 8, 1, 1, 2))]
    # (largest M, fm, fn, K-slices) per projection, best of tools/mid_gemm_bench.py on MI355X
    # (profiles/r2_mid_gemm_sweep.jsonl); the first row whose M covers the step is used
    # 32-row tiles (fm = 1) from profiles/r2_mid_fm1_sweep.jsonl: 2-16 % faster at 17-64 rows
    MID_CFG = {
        "qkv": [(32, 1, 2, 2), (64, 1, 2, 1), (128, 2, 2, 1), (256, 4, 2, 1), (1 << 30, 4, 4, 1)],
        "o": [(32, 1, 2, 4), (64, 1, 2, 2), (128, 2, 2, 2), (256, 2, 2, 1), (1 << 30, 4, 2, 1)],
        "gate_up": [(32, 1, 4, 1), (64, 2, 4, 1), (128, 4, 4, 1), (256, 8, 4, 1), (1 << 30, 8, 4, 1)],
        "down": [(32, 1, 2, 4), (64, 2, 2, 4), (128, 2, 2, 2), (256, 4, 2, 2), (1 << 30, 4, 4, 2)],
    }

    def __init__(self, cfg: LlamaConfig, device, dtype=torch.bfloat16, tp: Optional[TPGroup] = None,
                 seed: int = 0, weights_path: Optional[str] = None, decode_pack: Optional[bool] = None,
                 keep_dense: Optional[bool] = None):
        """keep_dense: keep the row-major projection weights after packing (None: only on CPU,
        where the tests read them). On the GPU the packed copy is the ONLY copy (VERDICT r5
        item 6: the row-major one was 15 GB of dead HBM on 8B and kept 70B at TP=1 off the hand
        kernels); the dense reference paths unpack a layer at a time on demand."""
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp = tp or TPGroup.single()
        # routing-table overrides for in-engine A/Bs (tools/midrange_ab.py style): a JSON object
        # {"STREAM_CFG": {"qkv": [[64, [1, 1, 6, 1, 4, 4]]]}, "MID_CFG": {...}, "PF_CFG": {...},
        #  "PF_MIDRANGE": ["gate_up", "qkv"]} whose per-projection rows replace the class table's
        # rows for that projection (PF_MIDRANGE: the whole set)
        ov = os.environ.get("PILOTTAI_ROUTING_JSON")
        if ov:
            import json

            for table, rows in json.loads(ov).items():
                if table == "PF_MIDRANGE":  # a list of projection kinds
                    self.PF_MIDRANGE = frozenset(rows)
                    continue
                if table not in ("STREAM_CFG", "MID_CFG", "PF_CFG"):
                    raise ValueError(f"PILOTTAI_ROUTING_JSON: unknown table {table!r}")
                merged = dict(getattr(self, table))
                for kind, r in rows.items():
                    merged[kind] = [tuple(x) if table == "MID_CFG" else
                                    (x[0], tuple(x[1])) if table == "STREAM_CFG" else (x[0], x[1], dict(x[2]))
                                    for x in r]
                setattr(self, table, merged)
        ts = self.tp.size
        if cfg.num_heads % ts or cfg.num_kv_heads % ts or cfg.intermediate_size % ts or cfg.vocab_size % ts:
            raise ValueError(f"{cfg.name} is not divisible by tensor-parallel size {ts}")
        self.h_local = cfg.num_heads // ts
        self.kv_local = cfg.num_kv_heads // ts
        self.f_local = cfg.intermediate_size // ts
        self.v_local = cfg.vocab_size // ts
        self.vocab_offset = self.tp.rank * self.v_local
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.cos_sin = ref.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta,
                                        cfg.rope_scaling).to(self.device)
        if weights_path:
            self._load_hf(weights_path)
        else:
            self._init_random(seed)
        self.decode_packed = False
        self.keep_dense = (self.device.type != "cuda") if keep_dense is None else bool(keep_dense)
        if decode_pack is None:
            decode_pack = self._pack_fits()
        if decode_pack:
            self._pack_decode_weights()

    # -- decode weight copies ------------------------------------------------------
    def _pack_fits(self) -> bool:
        """Packing replaces the row-major projections layer by layer (peak: the weights plus
        one layer's temporaries), so it fits whenever the weights leave room for the KV cache:
        Llama-3-8B (15 GB), 70B at TP=8 (17.6 GB per GPU) and at TP=1 (141 GB of 288). With
        keep_dense both copies must fit in 45 % of the card."""
        if self.device.type != "cuda":
            return True
        total = torch.cuda.get_device_properties(self.device).total_memory
        if self.keep_dense:
            return 2 * self.weight_bytes() <= 0.45 * total
        return self.weight_bytes() <= 0.7 * total

    def _pack_decode_weights(self):
        """Fragment-major copies for ops.decode_gemm, with the RMSNorm weights
        folded into the columns of the matrices they feed (QKV <- ln1, gate_up <-
        ln2), so the decode path needs no separate norm kernel."""
        for L in self.layers:
            L["wqkv_p"] = ops.pack_decode_qkv_rope(L["wqkv"] * L["ln1"][None, :])
            L["wo_p"] = ops.pack_decode_weight(L["wo"])
            L["w13_p"] = ops.pack_decode_gate_up(L["w13"] * L["ln2"][None, :])
            L["w2_p"] = ops.pack_decode_weight(L["w2"])
            if not self.keep_dense:  # the packed copy is the only one (freed layer by layer)
                for k in DENSE_KINDS:
                    del L[k]
        self.lm_head_p = ops.pack_decode_weight(self.lm_head)
        # the row-major LM head goes too when the prefill kernels take its shard (N % 256 == 0:
        # the vocabulary at TP = 1 / 8B and 70B); a TP shard of another width (128,256 / 8 =
        # 16,032) keeps it for the library GEMM of > 32-row steps (0.26 GB at 70B TP = 8)
        if not self.keep_dense and self.lm_head is not self.embed and self.lm_head.shape[0] % 256 == 0:
            self.lm_head = None
        if self.device.type == "cuda":
            ops.decode_workspace(self.device)  # split-K slabs + tickets, before any graph capture
            ops.mid_workspace(self.device)
            ops.prefill_workspace(self.device)
            ops.stream_workspace(self.device)
        # RMSNorm row statistics handed from each residual epilogue to the next projection
        self._ss = torch.zeros(2, 1 << 15, dtype=torch.float32, device=self.device)
        self.decode_packed = True

    def dense(self, L: Dict[str, torch.Tensor], kind: str) -> torch.Tensor:
        """Row-major [N, K] weight `kind` ("wqkv", "wo", "w13", "w2") of layer dict L: the kept
        copy, or unpacked from the packed one (the folded RMSNorm weight divided back out; exact
        for unit norm weights, the random-init case). Reference / test paths only."""
        w = L.get(kind)
        if w is not None:
            return w
        if kind == "wqkv":
            return (ops.unpack_decode_qkv_rope(L["wqkv_p"]).float() / L["ln1"].float()[None, :]).to(self.dtype)
        if kind == "w13":
            return (ops.unpack_decode_gate_up(L["w13_p"]).float() / L["ln2"].float()[None, :]).to(self.dtype)
        return ops.unpack_decode_weight(L[{"wo": "wo_p", "w2": "w2_p"}[kind]])

    def dense_lm_head(self) -> torch.Tensor:
        return self.lm_head if self.lm_head is not None else ops.unpack_decode_weight(self.lm_head_p)

    def _dense_needed(self, T: int) -> bool:
        return not self.decode_packed or T > max(self.MID_MAX_T, self.PREFILL_MAX_T)

    # -- weights -----------------------------------------------------------------
    def _init_random(self, seed: int):
        """Random init in canonical shards: every parallel matrix is generated as
        C = num_kv_heads chunks along its split dimension, chunk j from its own
        seed. TP=k rank r generates only its chunks, so any TP degree that divides
        C holds exactly the slices of the TP=1 weights (TP tests compare token for
        token), and no rank ever materialises a full matrix."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        C = cfg.num_kv_heads
        ts, r = self.tp.size, self.tp.rank
        if C % ts:
            raise ValueError(f"TP size {ts} must divide num_kv_heads={C}")
        mine = range(r * C // ts, (r + 1) * C // ts)
        std, d, hd = cfg.init_std, cfg.hidden_size, cfg.head_dim

        def chunk(tag: int, j: int, *shape):
            g = torch.Generator(device=dev)
            g.manual_seed((seed * 1_000_003 + tag * 7919 + j) & 0x7FFFFFFF)
            t = torch.empty(*shape, dtype=dt, device=dev)
            t.normal_(0.0, std, generator=g)
            return t

        def rows(tag, total_rows, cols):  # column-parallel: split the output rows
            return torch.cat([chunk(tag, j, total_rows // C, cols) for j in mine], 0)

        def colsplit(tag, rows_, total_cols):  # row-parallel: split the input columns
            return torch.cat([chunk(tag, j, rows_, total_cols // C) for j in mine], 1)

        self.embed = rows(1, cfg.vocab_size, d)
        self.layers: List[Dict[str, torch.Tensor]] = []
        for li in range(cfg.num_layers):
            t = 100 + 10 * li
            q = rows(t + 0, cfg.num_heads * hd, d)
            k = rows(t + 1, cfg.num_kv_heads * hd, d)
            v = rows(t + 2, cfg.num_kv_heads * hd, d)
            gate = rows(t + 4, cfg.intermediate_size, d)
            up = rows(t + 5, cfg.intermediate_size, d)
            self.layers.append({
                "ln1": torch.ones(d, dtype=dt, device=dev),
                "wqkv": torch.cat([q, k, v], 0),
                "wo": colsplit(t + 3, d, cfg.num_heads * hd),
                "ln2": torch.ones(d, dtype=dt, device=dev),
                "w13": torch.cat([gate, up], 0),
                "w2": colsplit(t + 6, d, cfg.intermediate_size),
            })
            del q, k, v, gate, up
        self.norm = torch.ones(d, dtype=dt, device=dev)
        self.lm_head = self.embed if cfg.tie_embeddings else rows(2, cfg.vocab_size, d)

    def _load_hf(self, path: str):
        """Load a HF Llama checkpoint directory of *.safetensors (no pickle)."""
        from safetensors import safe_open

        cfg, dev, dt = self.cfg, self.device, self.dtype
        files = sorted(f for f in os.listdir(path) if f.endswith(".safetensors"))
        tensors: Dict[str, torch.Tensor] = {}
        for f in files:
            with safe_open(os.path.join(path, f), framework="pt") as fh:
                for k in fh.keys():
                    tensors[k] = fh.get_tensor(k)
        r, ts, hd = self.tp.rank, self.tp.size, cfg.head_dim

        def rows(t, n):  # column-parallel shard of the output dim
            return t.chunk(ts, dim=0)[r] if ts > 1 else t

        def cols(t):  # row-parallel shard of the input dim
            return t.chunk(ts, dim=1)[r] if ts > 1 else t

        def get(k):
            return tensors[k].to(dt)

        self.embed = rows(get("model.embed_tokens.weight"), 0).to(dev)
        self.layers = []
        for i in range(cfg.num_layers):
            p = f"model.layers.{i}."
            q = rows(get(p + "self_attn.q_proj.weight"), 0)
            k = rows(get(p + "self_attn.k_proj.weight"), 0)
            v = rows(get(p + "self_attn.v_proj.weight"), 0)
            gate = rows(get(p + "mlp.gate_proj.weight"), 0)
            up = rows(get(p + "mlp.up_proj.weight"), 0)
            self.layers.append({
                "ln1": get(p + "input_layernorm.weight").to(dev),
                "wqkv": torch.cat([q, k, v], 0).contiguous().to(dev),
                "wo": cols(get(p + "self_attn.o_proj.weight")).contiguous().to(dev),
                "ln2": get(p + "post_attention_layernorm.weight").to(dev),
                "w13": torch.cat([gate, up], 0).contiguous().to(dev),
                "w2": cols(get(p + "mlp.down_proj.weight")).contiguous().to(dev),
            })
            del q, k, v, gate, up
        self.norm = get("model.norm.weight").to(dev)
        if "lm_head.weight" in tensors and not cfg.tie_embeddings:
            self.lm_head = rows(get("lm_head.weight"), 0).contiguous().to(dev)
        else:
            self.lm_head = self.embed
        _ = hd

    def weight_bytes(self) -> int:
        n = self.embed.numel() + self.norm.numel()
        if self.lm_head is not None and self.lm_head is not self.embed:
            n += self.lm_head.numel()
        if getattr(self, "lm_head_p", None) is not None:
            n += self.lm_head_p.numel()
        for L in self.layers:
            n += sum(t.numel() for t in L.values())
        return n * self.embed.element_size()

    # -- forward -----------------------------------------------------------------
    def _embed(self, ids: torch.Tensor) -> torch.Tensor:
        if self.tp.size == 1:
            return F.embedding(ids, self.embed)
        local = ids - self.vocab_offset
        ok = (local >= 0) & (local < self.v_local)
        h = F.embedding(local.clamp(0, self.v_local - 1), self.embed) * ok.unsqueeze(-1).to(self.dtype)
        self.tp.all_reduce(h)
        return h

    def forward(self, meta: StepMeta, kv: KVCache, num_tokens: int, num_logit_rows: int,
                part_o: torch.Tensor, part_ml: torch.Tensor, embed=None) -> torch.Tensor:
        """Returns local-vocab logits [num_logit_rows, V/tp] (bf16).

        embed = (rows [>= T] int32, pool [R + 1, d] fp32): every token's final-norm hidden
        state is added to pool[rows[t]] (embedding requests; row R collects the others)."""
        cfg = self.cfg
        T = num_tokens
        if self.decode_packed and T <= self.DECODE_FUSED_MAX_T:
            return self._forward_decode(meta, kv, T, num_logit_rows, part_o, part_ml, embed)
        if self.decode_packed and (T <= self.MID_MAX_T or T <= self.PREFILL_MAX_T):
            return self._forward_mid(meta, kv, T, num_logit_rows, part_o, part_ml, embed)
        H, KVh, hd = self.h_local, self.kv_local, cfg.head_dim
        if not self.keep_dense and self.decode_packed:
            raise RuntimeError(f"a {T}-token step needs the row-major weights, which were freed after packing: "
                               "build the model with keep_dense=True (EngineConfig.keep_dense) to run such steps "
                               "on the library GEMMs")
        ids = meta.input_ids[:T].long() if self.device.type == "cpu" else meta.input_ids[:T]
        h = self._embed(ids)
        resid = h
        x = ops.rmsnorm(h, self.layers[0]["ln1"], cfg.rms_eps)
        for li, L in enumerate(self.layers):
            qkv = ops.linear(x, L["wqkv"], "qkv")
            q = torch.empty(T, H, hd, dtype=self.dtype, device=self.device)
            ops.rope_cache(q, kv.k[li], kv.v[li], qkv, meta.positions, meta.slots, self.cos_sin, H, KVh)
            attn = torch.empty(T, H, hd, dtype=self.dtype, device=self.device)
            ops.paged_attention(attn, part_o, part_ml, q, kv.k[li], kv.v[li], meta.items, meta.n_items,
                                meta.att_counters, meta.q_start, meta.q_len, meta.ctx_len,
                                meta.block_table, self.scale, num_seqs=meta.num_seqs, part_size=meta.part_size)
            o = ops.linear(attn.view(T, H * hd), L["wo"], "o")
            if self.tp.size > 1:
                self.tp.all_reduce(o)
            x = ops.fused_add_rmsnorm(resid, o, L["ln2"], cfg.rms_eps)
            gu = ops.linear(x, L["w13"], "gate_up")
            a = ops.silu_mul(gu)
            d = ops.linear(a, L["w2"], "down")
            if self.tp.size > 1:
                self.tp.all_reduce(d)
            nxt = self.layers[li + 1]["ln1"] if li + 1 < len(self.layers) else self.norm
            x = ops.fused_add_rmsnorm(resid, d, nxt, cfg.rms_eps)
        if embed is not None:
            self._pool_embed(x, T, embed)
        rows = meta.logit_rows[:num_logit_rows]
        rows = rows.long() if self.device.type == "cpu" else rows
        xs = x.index_select(0, rows)
        return ops.linear(xs, self.lm_head, "lm_head")

    def _forward_decode(self, meta: StepMeta, kv: KVCache, T: int, num_logit_rows: int,
                        part_o: torch.Tensor, part_ml: torch.Tensor, embed=None) -> torch.Tensor:
        """Decode-sized step on the packed weights: 5 launches per layer
        (norm+QKV+RoPE+KV write, attention, O+residual, norm+gate_up+SwiGLU,
        down+residual) instead of 9; the residual stream h is updated in place."""
        cfg = self.cfg
        H, KVh, hd = self.h_local, self.kv_local, cfg.head_dim
        eps = cfg.rms_eps
        tp = self.tp.size > 1
        ids = meta.input_ids[:T].long() if self.device.type == "cpu" else meta.input_ids[:T]
        h = self._embed(ids)
        if not h.is_contiguous():
            h = h.contiguous()
        for li, L in enumerate(self.layers):
            q = torch.empty(T, H, hd, dtype=self.dtype, device=self.device)
            ops.decode_qkv_rope(h, L["wqkv_p"], eps, q, kv.k[li], kv.v[li], meta.positions, meta.slots,
                                self.cos_sin, H, KVh)
            attn = torch.empty(T, H, hd, dtype=self.dtype, device=self.device)
            ops.paged_attention(attn, part_o, part_ml, q, kv.k[li], kv.v[li], meta.items, meta.n_items,
                                meta.att_counters, meta.q_start, meta.q_len, meta.ctx_len,
                                meta.block_table, self.scale, num_seqs=meta.num_seqs, part_size=meta.part_size,
                                waves=self.ATT_DECODE_WAVES)
            a2 = attn.view(T, H * hd)
            if tp:  # all-reduce + residual add in one launch (custom_ar.hip RES epilogue)
                self.tp.all_reduce_add(ops.decode_gemm(a2, L["wo_p"], "plain"), h)
            else:
                ops.decode_gemm(a2, L["wo_p"], "resid", resid=h, out=h)
            a = ops.decode_gemm(h, L["w13_p"], "silu", norm=True, eps=eps)
            if tp:
                self.tp.all_reduce_add(ops.decode_gemm(a, L["w2_p"], "plain"), h)
            else:
                ops.decode_gemm(a, L["w2_p"], "resid", resid=h, out=h, **self._down_cfg(T))
        if embed is not None:
            self._pool_embed(ops.rmsnorm(h, self.norm, eps), T, embed)
        rows = meta.logit_rows[:num_logit_rows]
        rows = rows.long() if self.device.type == "cpu" else rows
        xs = ops.rmsnorm(h.index_select(0, rows), self.norm, eps)
        return ops.decode_gemm(xs, self.lm_head_p, "plain")

    @staticmethod
    def _down_cfg(T: int) -> dict:
        """down_proj config for decode steps: one 16-column tile x 8 waves per workgroup, no
        K split, at 8 and at 9-16 rows (cache-cold, interleaved: 21.0 us at M = 8, 25.4 us at
        M = 16 against 27.6 for the 2-tile x 16-wave x 2-slice config that 9-16-row steps
        used before; profiles/r3_decode_cfg_sweep.jsonl, tools/decode_cfg_sweep.py)."""
        return {"nt": 1, "waves": 8}

    @staticmethod
    def _pool_embed(hn: torch.Tensor, T: int, embed):
        """Sum each token's final-norm hidden state into its pooling row (graph-capturable)."""
        rows, pool = embed
        pool[-1].zero_()  # the row collecting non-embedding tokens holds one step's sums only
        pool.index_add_(0, rows[:T].long(), hn[:T].float())

    def _mid_cfg(self, kind: str, T: int) -> dict:
        for mmax, fm, fn, S in self.MID_CFG[kind]:
            if T <= mmax:
                return {"fm": fm, "fn": fn, "splits": S}
        return {}

    @staticmethod
    def _stream_plan(M: int, shape) -> tuple:
        """Full stream-kernel plan (mg, rg, tpw, wt, wk, S, D) for M rows from a table shape
        (rg, tpw, wt, wk, S, D): mg = the smallest instantiated row-fragment count (2, 4, 8)
        whose rg row groups cover M, with the row-group count closest to the table's for
        which every group holds rows (gemm_stream.hip plan_ok)."""
        rg0, tpw, wt, wk, S, D = (int(v) for v in shape)
        for rg in sorted(range(1, 17), key=lambda r: (abs(r - rg0), r)):
            need = -(-M // (16 * rg))
            mg = next((m for m in (2, 4, 8) if m >= need), 0)
            if mg and 16 * mg * (rg - 1) < M:
                return (mg, rg, tpw, wt, wk, S, D)
        raise ValueError(f"no stream plan for M={M} with shape {shape}")

    @staticmethod
    def _stream_plan_ok(plan, M: int, N: int, K: int, pair: bool) -> bool:
        """Host mirror of gemm_stream.hip plan_ok (+ the workspace bound), so a table row that
        does not fit a shape falls back instead of failing at launch."""
        mg, rg, tpw, wt, wk, S, D = plan
        tiles, KS, CT = N // 16, K // 32, tpw * wt
        if N % 16 or K % 64 or tiles % CT or (pair and CT % 2) or KS % S or (KS // S) % (2 * wk):
            return False
        nch = KS // S // (2 * wk)
        if nch < D or nch % D or 16 * mg * rg < M or 16 * mg * (rg - 1) >= M:
            return False
        grid = tiles // CT * rg * S
        if S > 1 and grid > 256:
            return False
        from pilottai_amd.ops import kernels

        direct = S * wk == 1 and (not pair or tpw % 2 == 0)  # no slabs (gemm_stream.hip)
        return direct or (tiles // CT) * rg * S * wk * CT * mg * 256 <= kernels.STREAM_WS_FLOATS

    def _stream_for(self, kind: str, T: int, N: int, K: int, rows, pair: bool = False):
        nk = self.STREAM_NK.get(kind)
        if nk is not None and tuple(nk) != (N, K):
            return None
        for mmax, shape in rows:
            if T <= mmax:
                try:
                    plan = self._stream_plan(T, shape)
                except ValueError:
                    return None
                return plan if self._stream_plan_ok(plan, T, N, K, pair) else None
        return None

    def _proj_path(self, kind: str, T: int, N: int = 0, K: int = 0):
        """("stream" | "mid" | "pf", cfg) for projection `kind` (N x K weights) on a T-token step."""
        if T <= self.MID_MAX_T and N:
            plan = self._stream_for(kind, T, N, K, self.STREAM_CFG.get(kind, ()),
                                    pair=kind in ("qkv", "gate_up"))
            if plan is not None:
                return "stream", {"plan": plan}
        if self.device.type == "cuda" and (T > self.MID_MAX_T or kind in self.PF_MIDRANGE):
            for mmax, path, cfg in self.PF_CFG[kind]:
                if T <= mmax:
                    if path != "pf":
                        return path, self._mid_cfg(kind, T) | dict(cfg)
                    cfg = dict(cfg)
                    if cfg.get("bn") == 192 and N % 192:  # 256 x 192 tiles need N % 192 == 0
                        cfg["bn"] = 256
                    return path, cfg
        return "mid", self._mid_cfg(kind, T)

    def _gemm(self, kind: str, T: int, x, wp, epi: str, **kw):
        path, cfg = self._proj_path(kind, T, wp.shape[0] * 16, wp.shape[1] * 32)
        fn = {"pf": ops.prefill_gemm, "stream": ops.stream_gemm}.get(path, ops.mid_gemm)
        return fn(x, wp, epi, **cfg, **kw)

    def _qkv_rope(self, T: int, x, wp, eps, q, k_cache, v_cache, meta, ss_in):
        H, KVh = self.h_local, self.kv_local
        if T <= min(self.DEC_QKV_MAX_T, 64) and self.device.type == "cuda":
            return ops.decode_qkv_rope(x, wp, eps, q, k_cache, v_cache, meta.positions, meta.slots, self.cos_sin,
                                       H, KVh)
        path, cfg = self._proj_path("qkv", T, wp.shape[0] * 16, wp.shape[1] * 32)
        fn = {"pf": ops.prefill_qkv_rope, "stream": ops.stream_qkv_rope}.get(path, ops.mid_qkv_rope)
        return fn(x, wp, eps, q, k_cache, v_cache, meta.positions, meta.slots, self.cos_sin, H, KVh,
                  ss_in=ss_in, **cfg)

    def _forward_mid(self, meta: StepMeta, kv: KVCache, T: int, num_logit_rows: int,
                     part_o: torch.Tensor, part_ml: torch.Tensor, embed=None) -> torch.Tensor:
        """Mid-size and prefill-heavy steps (T > DECODE_FUSED_MAX_T: decode rows plus prefill chunks)
        on the packed weights, 4 projection launches + attention per layer
        (csrc/ops/gemm_mid.hip up to MID_MAX_T tokens; above it the 256 x 256 tiles of
        csrc/ops/gemm_prefill.hip for the projections PF_CFG assigns to them):

          QKV (RMSNorm folded, RoPE + paged KV write in the epilogue) -> attention ->
          O (+ residual, accumulating the next norm's row statistics) ->
          gate_up (RMSNorm folded, SwiGLU epilogue) -> down (+ residual, statistics)

        The RMSNorm statistics sum(h^2) of each row are produced by the residual epilogue
        that writes h (buffers ss_a / ss_b alternate; each residual launch zeroes the
        buffer the next one fills), so no norm kernel runs. Under TP the row-parallel
        outputs go through TPGroup.all_reduce_add: all-reduce, residual add and the row
        statistics in one custom all-reduce launch (RCCL + add + row_sumsq as the fallback)."""
        cfg = self.cfg
        H, KVh, hd = self.h_local, self.kv_local, cfg.head_dim
        eps = cfg.rms_eps
        tp = self.tp.size > 1
        ids = meta.input_ids[:T].long() if self.device.type == "cpu" else meta.input_ids[:T]
        h = self._embed(ids)
        if not h.is_contiguous():
            h = h.contiguous()
        ss_a, ss_b = self._ss[0, :T], self._ss[1, :T]
        ops.row_sumsq(h, out=ss_a)
        ss_b.zero_()
        for li, L in enumerate(self.layers):
            q = torch.empty(T, H, hd, dtype=self.dtype, device=self.device)
            self._qkv_rope(T, h, L["wqkv_p"], eps, q, kv.k[li], kv.v[li], meta, ss_a)
            attn = torch.empty(T, H, hd, dtype=self.dtype, device=self.device)
            ops.paged_attention(attn, part_o, part_ml, q, kv.k[li], kv.v[li], meta.items, meta.n_items,
                                meta.att_counters, meta.q_start, meta.q_len, meta.ctx_len,
                                meta.block_table, self.scale, num_seqs=meta.num_seqs, part_size=meta.part_size,
                                waves=self.ATT_MID_WAVES)
            a2 = attn.view(T, H * hd)
            if tp:  # all-reduce + residual + the next norm's row statistics in one launch;
                # ss_b was zeroed by the previous down all-reduce (or above), ss_a is zeroed here
                self.tp.all_reduce_add(self._gemm("o", T, a2, L["wo_p"], "plain"), h, ss=ss_b, ss_zero=ss_a)
            else:  # ss_b was zeroed by the previous down launch (or above)
                self._gemm("o", T, a2, L["wo_p"], "resid", resid=h, out=h, ss_out=ss_b, ss_zero=ss_a)
            a = self._gemm("gate_up", T, h, L["w13_p"], "silu", norm=True, eps=eps, ss_in=ss_b)
            if tp:
                self.tp.all_reduce_add(self._gemm("down", T, a, L["w2_p"], "plain"), h, ss=ss_a, ss_zero=ss_b)
            else:
                self._gemm("down", T, a, L["w2_p"], "resid", resid=h, out=h, ss_out=ss_a, ss_zero=ss_b)
        if embed is not None:
            self._pool_embed(ops.rmsnorm(h, self.norm, eps), T, embed)
        rows = meta.logit_rows[:num_logit_rows]
        rows = rows.long() if self.device.type == "cpu" else rows
        xs = ops.rmsnorm(h.index_select(0, rows), self.norm, eps)
        return self._lm_head(xs, num_logit_rows)

    def _lm_head(self, xs, n: int):
        """Logits of the step's sampling rows on the packed weights: the weight-streaming kernel
        where LM_HEAD_STREAM covers n (> 16 rows), else the packed decode kernel up to 32 rows,
        else hipBLASLt."""
        if n > self.DECODE_FUSED_MAX_T:
            wp = self.lm_head_p
            plan = self._stream_for("lm_head", n, wp.shape[0] * 16, wp.shape[1] * 32, self.LM_HEAD_STREAM)
            if plan is not None:
                return ops.stream_gemm(xs, wp, "plain", plan=plan)
        if n <= 32:
            return ops.decode_gemm(xs, self.lm_head_p, "plain")
        if self.lm_head is None:  # packed only: the prefill kernels take any row count
            return ops.prefill_gemm(xs, self.lm_head_p, "plain")
        return ops.linear(xs, self.lm_head, "lm_head")

    # -- reference (dense, no cache) forward used by numerics tests ----------------
    @torch.no_grad()
    def reference_logits(self, token_ids: List[int]) -> torch.Tensor:
        """Plain PyTorch fp32-math causal forward over one sequence (TP=1 only)."""
        assert self.tp.size == 1
        cfg = self.cfg
        T = len(token_ids)
        ids = torch.tensor(token_ids, device=self.device)
        h = F.embedding(ids, self.embed).float()
        pos = torch.arange(T, device=self.device)
        H, KVh, hd = self.h_local, self.kv_local, cfg.head_dim
        mask = torch.full((T, T), float("-inf"), device=self.device).triu(1)
        for L0 in self.layers:
            L = {k: self.dense(L0, k) for k in DENSE_KINDS}
            L["ln1"], L["ln2"] = L0["ln1"], L0["ln2"]
            x = ref.rmsnorm(h.to(self.dtype), L["ln1"], cfg.rms_eps).float()
            qkv = (x.to(self.dtype).float() @ L["wqkv"].float().T).to(self.dtype)
            q = ref.apply_rope(qkv[:, :H * hd].view(T, H, hd), pos, self.cos_sin)
            k = ref.apply_rope(qkv[:, H * hd:(H + KVh) * hd].view(T, KVh, hd), pos, self.cos_sin)
            v = qkv[:, (H + KVh) * hd:].view(T, KVh, hd)
            G = H // KVh
            kh = k.float().repeat_interleave(G, 1).permute(1, 0, 2)
            vh = v.float().repeat_interleave(G, 1).permute(1, 0, 2)
            s = (q.float().permute(1, 0, 2) @ kh.transpose(1, 2)) * self.scale + mask
            o = (torch.softmax(s, -1) @ vh).permute(1, 0, 2).reshape(T, H * hd).to(self.dtype)
            h = (h.to(self.dtype).float() + (o.float() @ L["wo"].float().T).to(self.dtype).float())
            x = ref.rmsnorm(h.to(self.dtype), L["ln2"], cfg.rms_eps)
            gu = (x.float() @ L["w13"].float().T).to(self.dtype)
            a = ref.silu_mul(gu)
            h = (h.to(self.dtype).float() + (a.float() @ L["w2"].float().T).to(self.dtype).float())
        x = ref.rmsnorm(h.to(self.dtype), self.norm, cfg.rms_eps)
        return (x.float() @ self.dense_lm_head().float().T)

    # -- dense batched encoder forward (semantic-memory embeddings) ----
    @torch.no_grad()
    def hidden_states(self, batch: List[List[int]], pooling: str = "mean") -> torch.Tensor:
        """Final-norm hidden states mean-pooled over each sequence's tokens (pooling="last":
        the state of each sequence's last token): [B, d].

        A dense bf16 causal forward (library GEMMs + SDPA attention, no KV cache),
        right-padded to the longest sequence; used by EngineEmbedder to embed
        memory items with the serving model itself. TP=1 only."""
        assert self.tp.size == 1, "hidden_states runs on a TP=1 model"
        cfg, dev, dt = self.cfg, self.device, self.dtype
        B = len(batch)
        T = max(1, max(len(s) for s in batch))
        ids = torch.zeros(B, T, dtype=torch.long, device=dev)
        valid = torch.zeros(B, T, dtype=torch.bool, device=dev)
        for i, s in enumerate(batch):
            if s:
                ids[i, :len(s)] = torch.tensor(s, device=dev)
                valid[i, :len(s)] = True
        H, KVh, hd = self.h_local, self.kv_local, cfg.head_dim
        pos = torch.arange(T, device=dev)
        cs = self.cos_sin[:T]
        cos, sin = cs[:, : hd // 2].to(dt), cs[:, hd // 2:].to(dt)

        def rope(x):  # [B, T, h, hd], rotate-half
            x1, x2 = x[..., : hd // 2], x[..., hd // 2:]
            c, s = cos[None, :, None, :], sin[None, :, None, :]
            return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)

        h = F.embedding(ids, self.embed)                      # [B, T, d]
        for L0 in self.layers:
            L = {k: self.dense(L0, k) for k in DENSE_KINDS}
            x = F.rms_norm(h, (cfg.hidden_size,), L0["ln1"], cfg.rms_eps)
            qkv = F.linear(x, L["wqkv"])
            q = rope(qkv[..., : H * hd].view(B, T, H, hd))
            k = rope(qkv[..., H * hd:(H + KVh) * hd].view(B, T, KVh, hd))
            v = qkv[..., (H + KVh) * hd:].view(B, T, KVh, hd)
            o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                               is_causal=True, enable_gqa=True, scale=self.scale)
            h = h + F.linear(o.transpose(1, 2).reshape(B, T, H * hd), L["wo"])
            x = F.rms_norm(h, (cfg.hidden_size,), L0["ln2"], cfg.rms_eps)
            gu = F.linear(x, L["w13"])
            g, u = gu.chunk(2, dim=-1)
            h = h + F.linear(F.silu(g) * u, L["w2"])
        x = F.rms_norm(h, (cfg.hidden_size,), self.norm, cfg.rms_eps).float()
        if pooling == "last":
            last = torch.tensor([max(1, len(s)) - 1 for s in batch], device=dev)
            return x[torch.arange(B, device=dev), last]
        w = valid.unsqueeze(-1).float()
        return (x * w).sum(1) / w.sum(1).clamp_min(1.0)
