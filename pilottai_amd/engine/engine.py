"""On-node LLM inference engine (replaces the reference's remote litellm provider,
pilott/engine/llm.py:12-219, with a local Llama-3 on MI355X).

Architecture (one engine per GPU / per TP group, one process per GPU):

    asyncio agents ──submit()──► inbox ──► engine thread ──► native Scheduler (C++)
                                                  │   schedule(): writes the whole step into a
                                                  │   pinned int32 buffer (ids, positions, KV slots,
                                                  │   block tables, attention items, sampling params)
                                                  ▼
                        one H2D copy ─► hipGraph replay of [embed → 32 x layer → LM head → sample]
                                                  │   captured per token bucket (ragged batches of
                                                  │   decode + prefill + grammar jump-forward tokens)
                                                  ▼
                        sampled ids ─► Scheduler.commit(): grammar advance, jump-forward, stops,
                                       prefix-cache registration ─► completion callbacks

The LLM protocol used by agents (generate_response / apredict) lives in
engine/local_llm.py on top of `LLMEngine.submit`.

Tensor parallelism (Llama-3-70B, TP=8 over xGMI): only TP rank 0 (the driver)
owns requests, the scheduler, grammars and the tokenizer. Each step it sends a
7-int header over a gloo group, then broadcasts the step metadata it already
holds on the device (one RCCL broadcast); the other ranks sit in `follow()`,
replay the same hipGraph, and take part in the row-parallel all-reduces and
the vocab-parallel sampling collectives inside it (all-gather of per-shard winners; top-k /
top-p thresholds from all-reduced radix histograms, engine/tp_sampling.py). Their schedulers stay idle, so
nothing on the host has to be kept consistent between ranks.
"""
from __future__ import annotations

import logging
import os
import queue
import sys
from collections import deque
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, Union

import numpy as np
import torch

from pilottai_amd import ops
from pilottai_amd.engine.tp_sampling import tp_topkp_threshold
from pilottai_amd.models.llama import KVCache, LlamaModel, StepMeta, get_config
from pilottai_amd.parallel.comm import TPGroup
from pilottai_amd.utils.tracing import trace_range

from .grammar import MAX_CLASSES, GrammarCompiler
from .tokenizer import Tokenizer, get_tokenizer

log = logging.getLogger("pilottai_amd.engine")

# hipGraph token buckets: a step of T tokens replays the smallest bucket >= T, so
# the spacing bounds the padded (wasted) work: 16-token steps up to 512 (graph padding 1.9 ->
# 1.1 % of step tokens at 64 workers; profiles/r2_buckets16_ab.jsonl), 64 up to 2048
# (prefill-heavy agent steps sit at 400-1000 tokens).
DEFAULT_BUCKETS = ([8, 16, 32, 48, 64, 80] + list(range(96, 513, 16)) + list(range(576, 2049, 64))
                   + [3072, 4096, 6144, 8192])


@dataclass
class EngineConfig:
    model: str = "llama-3-8b"
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 2048
    max_prefill_tokens: int = 2048
    max_model_len: int = 8192
    block_size: int = 16
    num_kv_blocks: Optional[int] = None
    kv_cache_gb: Optional[float] = None
    kv_cache_fraction: float = 0.5
    kv_reserve_gb: float = 20.0  # HBM always left outside the KV pool (graphs, activations, workspaces)
    prefix_caching: bool = True
    dedup_inflight_prefix: bool = True  # requests wait for an identical prefix another request is prefilling
    # waiting embedding requests are admitted before waiting generation prompts (scheduler.h)
    embed_first: bool = os.environ.get("PILOTTAI_EMBED_FIRST", "1") != "0"
    split_decode: bool = True
    # > 0: mid / large steps size their decode partitions for about this many (partition, KV
    # head) workgroups (scheduler.h decode_part_target): no split once the decode rows fill a
    # round of 4-wave attention workgroups (2 per CU), equal partitions otherwise; 0 = the
    # 512 / 256-key partitions. 32 / 64 / 128-row steps (ctx 600) 4.10 / 4.87 / 5.54 ->
    # 4.05 / 4.67 / 5.45 ms (profiles/r4_att_mid_options_ab.jsonl); headline bench, same box:
    # 1,024 2 % worse than 512, 384 1 % better (profiles/r4_engine_knobs_ab.jsonl)
    decode_part_target: int = int(os.environ.get("PILOTTAI_DECODE_PART_TARGET", "384"))
    # decode-sized steps on 8-wave attention (scheduler.h small_step_part): the smallest
    # flash-decoding partition they use; 4096 = whole contexts (no merge) up to 4,096 keys
    small_step_part: int = int(os.environ.get("PILOTTAI_SMALL_STEP_PART", "4096"))
    # > 0: decode-sized steps size their partitions for about this many (partition, KV head)
    # 8-wave workgroups (scheduler.h small_step_target); 0 = small_step_part alone. 8-row steps
    # (ctx 600 / 1,200) 3.228 / 3.461 -> 3.172 / 3.331 ms, 16 rows unchanged
    # (profiles/r4_small_step_partitions_ab.jsonl)
    small_step_target: int = int(os.environ.get("PILOTTAI_SMALL_STEP_TARGET", "192"))
    use_graphs: bool = True
    token_buckets: Optional[List[int]] = None
    seed: int = 0
    weights_path: Optional[str] = None
    capture_on_start: bool = True
    token_align: int = 256   # GEMM-friendly step sizes (runtime/scheduler.h); 0 = off
    align_slack: int = 96
    decode_fused: Optional[bool] = None  # packed-weight fused decode path; None = when it fits in HBM
    decode_fused_max_t: Optional[int] = None  # largest step (tokens) on that path; None = model default
    mid_max_t: Optional[int] = None  # largest step on the LDS-DMA tiled mid-size path; None = model default
    # largest step on the fused packed-weight path with the 256 x 256 prefill kernels (above
    # mid_max_t); 0 = such steps take the library (hipBLASLt) path; None = model default
    prefill_max_t: Optional[int] = None
    # keep the row-major projection weights beside the packed ones (None: only when some step can
    # leave the packed-weight path, i.e. prefill_max_t / mid_max_t below max_num_batched_tokens)
    keep_dense: Optional[bool] = None
    # projections ("qkv", "o", "gate_up", "down") whose PF_CFG prefill-kernel rows also apply to
    # <= 256-token steps (None: model default)
    pf_midrange: Optional[List[str]] = None
    # LlamaModel class-level tunables to override on this engine's model (name -> value),
    # e.g. {"DEC_QKV_MAX_T": 64}; for A/B tools (tools/engine_ab.py)
    model_overrides: Optional[Dict[str, Any]] = None
    att_qcols: int = 128  # prefill attention item width in MFMA columns (128: LDS-staged 4-wave items)
    # ... used only for steps with at least this many prefill tokens (1,024: 1,024-2,048-token steps
    # 1-2 % faster than with 2,048, which most mixed steps never reached; profiles/r2_att_wide_min_ab.jsonl)
    att_wide_min_tokens: int = 1024
    # wide prefill items of at least this many causal keys are split into partitions merged
    # in-kernel (scheduler.h prefill_split_keys); 0 = off, the default: the wide path runs only
    # on steps whose items already fill the chip's 2 x 256 workgroup slots, where a split adds a
    # second round (profiles/r6_attention_split.md: 2,048-token prompt 69.7 -> 97.9 us at 512);
    # on few long items narrow items beat wide + split (cont256x4096: 32.4 vs 55.4 us)
    prefill_split_keys: int = int(os.environ.get("PILOTTAI_PREFILL_SPLIT_KEYS", "0"))
    # attention workgroup width on decode-sized steps (<= the model's DECODE_FUSED_MAX_T
    # tokens): 8 waves stream a whole context per workgroup (the scheduler then skips the
    # flash-decoding split for such steps when they have few rows); None = model default
    att_decode_waves: Optional[int] = None
    reply_tokens: Optional[int] = None  # fixed length of every reply schema's free-text slot (grammar.py)
    # interpreter thread-switch interval while the engine thread runs (sys.setswitchinterval);
    # None = env PILOTTAI_GIL_SWITCH_S or the interpreter default (5 ms)
    gil_switch_interval: Optional[float] = None
    # pipelined steps: step N+1 is scheduled and launched while step N runs;
    # rows sampling in N continue speculatively (runtime/scheduler.h). TP = 1 only.
    async_steps: bool = False
    # start(): gc.freeze() everything alive (model, graphs, tokenizer) so later cyclic
    # collections skip it (a full pass stalled the engine thread 60-85 ms). PROCESS-GLOBAL:
    # frozen objects are never reclaimed by the cycle collector until stop() unfreezes, so it
    # is opt-in, for serving entry points that build one engine (bench.py freezes after its
    # warm-up instead; the HTTP server sets it)
    freeze_heap: bool = False
    # keep every captured hipGraph's node list (torch keep_graph=True) so tools can count its
    # kernels (utils/tracing.py graph_node_counts); costs host memory, off in serving
    keep_graphs: bool = False


# TP step header: [op, T, ns, nsamp, bucket, masks_changed, n_copy, truncate, embed]
_OP_STOP, _OP_STEP = 0, 1


@dataclass
class GenerationOutput:
    request_id: int
    token_ids: List[int]
    finish_reason: str
    prompt_tokens: int
    cached_prompt_tokens: int
    completion_tokens: int
    sampled_tokens: int
    forced_tokens: int
    t_arrival: float
    t_first_token: float
    t_finish: float
    _tok: Optional[Tokenizer] = field(default=None, repr=False)
    embedding: Optional[np.ndarray] = field(default=None, repr=False)  # embedding requests: mean final hidden

    @property
    def text(self) -> str:
        return self._tok.decode(self.token_ids) if self._tok else ""

    @property
    def ttft(self) -> float:
        return max(0.0, self.t_first_token - self.t_arrival) if self.t_first_token > 0 else 0.0

    @property
    def latency(self) -> float:
        return max(0.0, self.t_finish - self.t_arrival)


_REASONS = {0: "stop", 1: "length", 2: "abort", 3: "embed"}


@dataclass
class _Request:
    rid: int
    prompt_ids: List[int]
    temperature: float
    max_tokens: int
    seed: int
    ignore_eos: bool
    stop_ids: List[int]
    grammar: Optional[list]
    callback: Callable[[GenerationOutput], None]
    t_arrival: float
    top_k: int = 0
    top_p: float = 1.0
    embed: bool = False
    embed_last: bool = False  # last-token pooling (prefix-cache reuse allowed)


class LLMEngine:
    def __init__(self, cfg: Optional[EngineConfig] = None, device=None, tp: Optional[TPGroup] = None,
                 tokenizer: Optional[Tokenizer] = None):
        from pilottai_amd import _runtime

        self._rt = _runtime
        self.cfg = cfg = cfg or EngineConfig()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.device = torch.device(device)
        self.on_gpu = self.device.type == "cuda"
        if self.on_gpu:
            ops.require_native()
            torch.cuda.set_device(self.device)
        self.tp = tp or TPGroup.single()
        self.tok = tokenizer or get_tokenizer()
        self.grammar = GrammarCompiler(self.tok, reply_tokens=cfg.reply_tokens)
        self.model_cfg = get_config(cfg.model)
        mc = self.model_cfg
        if self.on_gpu:
            from .gemm_tuning import load_tuned_gemms

            self.tuned_gemms = load_tuned_gemms(mc.name, self.tp.size)
        t0 = time.time()
        keep_dense = cfg.keep_dense
        if keep_dense is None and (cfg.prefill_max_t is not None or cfg.mid_max_t is not None):
            lim = max(LlamaModel.MID_MAX_T if cfg.mid_max_t is None else int(cfg.mid_max_t),
                      LlamaModel.PREFILL_MAX_T if cfg.prefill_max_t is None else int(cfg.prefill_max_t))
            keep_dense = True if lim < cfg.max_num_batched_tokens else None
        self.model = LlamaModel(mc, self.device, tp=self.tp, seed=cfg.seed, weights_path=cfg.weights_path,
                                decode_pack=cfg.decode_fused, keep_dense=keep_dense)
        if cfg.decode_fused_max_t is not None:
            self.model.DECODE_FUSED_MAX_T = int(cfg.decode_fused_max_t)
        if cfg.mid_max_t is not None:
            self.model.MID_MAX_T = int(cfg.mid_max_t)
        if cfg.prefill_max_t is not None:
            self.model.PREFILL_MAX_T = int(cfg.prefill_max_t)
        for k, v in (cfg.model_overrides or {}).items():
            if not hasattr(self.model, k):
                raise ValueError(f"unknown model tunable {k!r}")
            setattr(self.model, k, frozenset(v) if isinstance(getattr(self.model, k), frozenset) else v)
        if cfg.att_decode_waves is not None:
            self.model.ATT_DECODE_WAVES = int(cfg.att_decode_waves)
        if cfg.pf_midrange is not None:
            self.model.PF_MIDRANGE = frozenset(cfg.pf_midrange)
        self.load_time = time.time() - t0
        self.max_model_len = min(cfg.max_model_len, mc.max_position)
        # ---- KV cache sizing (288 GB HBM: the default leaves room for graphs/activations)
        kv_local = self.model.kv_local
        bpb = KVCache.bytes_per_block(mc.num_layers, kv_local, cfg.block_size)
        nb = cfg.num_kv_blocks
        if nb is None:
            if cfg.kv_cache_gb is not None:
                nb = int(cfg.kv_cache_gb * (1 << 30)) // bpb
            elif self.on_gpu:
                free, _total = torch.cuda.mem_get_info(self.device)
                # a fraction of what is free, but never into the reserve: beside a 205 GB
                # memory index (config 4) 15 % of the rest is too little for the graphs
                nb = int(max(0.0, min(free * cfg.kv_cache_fraction, free - cfg.kv_reserve_gb * (1 << 30)))) // bpb
            else:
                nb = 2048
        need_min = (self.max_model_len + cfg.block_size - 1) // cfg.block_size + 1
        nb = max(nb, need_min)
        if self.tp.size > 1:  # block ids travel in the metadata: every rank needs the same pool
            t = torch.tensor([nb], dtype=torch.int64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN, group=self.tp.cpu_group)
            nb = int(t.item())
        self.kv = KVCache(mc.num_layers, nb, kv_local, self.device, block_size=cfg.block_size)
        self.num_kv_blocks = nb
        # ---- native scheduler + step buffers
        # the model runs 8-wave decode attention on the fused decode path only, keyed on the
        # graph bucket: the scheduler's whole-context (unsplit) items for small steps must
        # follow the same rule, keyed on the step size -> the largest bucket on that path
        buckets = cfg.token_buckets or DEFAULT_BUCKETS
        self.buckets = sorted({b for b in buckets if b <= cfg.max_num_batched_tokens} |
                              {cfg.max_num_batched_tokens})
        small = [b for b in self.buckets if b <= self.model.DECODE_FUSED_MAX_T]
        small_step = max(small) if (small and self.model.ATT_DECODE_WAVES == 8 and self.model.decode_packed) else 0
        self.sched = _runtime.Scheduler({
            "num_blocks": nb, "block_size": cfg.block_size, "max_num_seqs": cfg.max_num_seqs,
            "max_num_batched_tokens": cfg.max_num_batched_tokens,
            "max_prefill_tokens": cfg.max_prefill_tokens, "max_model_len": self.max_model_len,
            "gqa_group": self.model.h_local // self.model.kv_local,
            "att_qcols": cfg.att_qcols,
            "att_wide_min_tokens": cfg.att_wide_min_tokens,
            "prefill_split_keys": cfg.prefill_split_keys,
            "prefix_caching": cfg.prefix_caching, "split_decode": cfg.split_decode,
            "dedup_inflight_prefix": cfg.dedup_inflight_prefix,
            "embed_first": bool(cfg.embed_first),
            "token_align": cfg.token_align, "align_slack": cfg.align_slack,
            "kv_heads": self.model.kv_local,
            "small_step_tokens": small_step,
            "small_step_part": int(cfg.small_step_part) if small_step else 0,
            "small_step_target": int(cfg.small_step_target) if small_step else 0,
            "decode_part_target": int(cfg.decode_part_target),
            "eos_ids": list(self.tok.eos_ids)})
        L = self.L = self.sched.layout()
        pin = self.on_gpu
        # pipelined steps: two host-side step descriptions (one being copied / in flight,
        # one being scheduled); the device copy is stream-ordered behind the previous step
        self._async = bool(cfg.async_steps) and self.tp.size == 1
        nbuf = 2 if self._async else 1
        self._host_metas = [torch.zeros(L["total"], dtype=torch.int32, pin_memory=pin) for _ in range(nbuf)]
        self._host_meta = self._host_metas[0]
        self._host_ptr = self._host_meta.data_ptr()
        self._host_np = self._host_meta.numpy()
        self._dev_meta = torch.zeros(L["total"], dtype=torch.int32, device=self.device) \
            if (self.on_gpu or self._async) else self._host_meta
        # attention tickets: one per (sequence, KV head) for split decode rows, then -- only with
        # prefill_split_keys on -- one per (partial slot, KV head) for split prefill items
        # (csrc/ops/attention.hip prefill_item_wg). Without that room the kernel runs its
        # instantiation with the partition hand-off compiled out (no register spills).
        pf_slots = L["max_items"] if cfg.prefill_split_keys > 0 else 0
        self._att_counters = torch.zeros((L["max_seqs"] + pf_slots) * kv_local, dtype=torch.int32,
                                         device=self.device)
        self._init_views()
        V = mc.vocab_size
        self._mask_words = (V + 31) // 32
        self._class_masks = torch.zeros(MAX_CLASSES, self._mask_words, dtype=torch.int32, device=self.device)
        self._mask_version = -1
        self._sync_masks()
        S = cfg.max_num_seqs
        S4 = (S + 3) & ~3  # the TP winners' all-gather moves 16-byte vectors (custom_ar.hip co_kernel)
        self._sampled_dev = torch.zeros(S4, dtype=torch.int32, device=self.device)
        self._sampled_hosts = [torch.zeros(S, dtype=torch.int32, pin_memory=pin) for _ in range(nbuf)]
        self._sampled_host = self._sampled_hosts[0]
        self._inflight: "deque" = deque()  # launched, not yet committed steps (pipelined mode)
        self._slot = 0
        self._last_done = 0.0
        self._keys_dev = torch.zeros(S4, dtype=torch.float32, device=self.device)
        # TP top-k / top-p: workspace of the HIP phase kernels (engine/tp_sampling.py)
        self._tkp_ws = None
        if self.tp.size > 1 and self.on_gpu:
            from .tp_sampling import tkp_ws_floats

            self._tkp_ws = torch.empty(tkp_ws_floats(S), dtype=torch.float32, device=self.device)
        # embedding requests: per-request pooling rows (+ one row that collects every other
        # token), summed in the step graph, read and cleared when the request finishes
        self._embed_pool = torch.zeros(L["max_seqs"] + 1, mc.hidden_size, dtype=torch.float32, device=self.device)
        self._embed_rows = self._dev_meta[L["embed_rows"]:L["embed_rows"] + L["max_tokens"]]
        # pipelined steps: a stream-ordered snapshot of the pool per step slot, taken right
        # behind the step that pools into it, so the commit reads host memory instead of
        # waiting (.cpu()) for the step queued after it
        self._embed_hosts = [torch.zeros_like(self._embed_pool, device="cpu", pin_memory=self.on_gpu)
                             for _ in range(2)] if self._async else None
        tpw = 16 // (self.model.h_local // self.model.kv_local)
        self._tpw = tpw
        self._max_parts = (self.max_model_len + ops.ATT_PART - 1) // ops.ATT_PART
        max_items = L["max_items"]
        # attention partition partials: written and merged inside one launch -> uncached memory
        self._part_o = ops.empty_handoff(max_items * kv_local * 16 * 128, torch.float32, self.device)
        self._part_ml = ops.empty_handoff(max_items * kv_local * 16 * 2, torch.float32, self.device)
        self._sample_ws = ops.sample_workspace(S, self.model.v_local, self.device) if self.on_gpu else None
        # one graph per (token bucket, top-k/top-p pass); truncating variants are
        # captured on first use, so steps without truncation pay nothing for it
        self._graphs: Dict[tuple, "torch.cuda.CUDAGraph"] = {}
        self._tau = torch.empty(S, dtype=torch.float32, device=self.device)
        self._graph_pool = None
        self.use_graphs = cfg.use_graphs and self.on_gpu
        if self.use_graphs and self.tp.size > 1 and getattr(self.tp, "custom", None) is None:
            # a TP step graph would capture RCCL collectives; every TP collective of a step
            # (activations, sampling winners, threshold histograms) needs the custom P2P path
            log.warning("TP=%d without the custom P2P collectives: running the steps eagerly", self.tp.size)
            self.use_graphs = False
        self.is_driver = self.tp.rank == 0
        self._tp_header = torch.zeros(9, dtype=torch.int64)
        self._tp_closed = False
        # ---- request plumbing
        self._inbox: "queue.SimpleQueue" = queue.SimpleQueue()
        self._aborts: "queue.SimpleQueue" = queue.SimpleQueue()
        self._wake = threading.Event()
        self._reqs: Dict[int, _Request] = {}
        self._pending_out: list = []  # finished outputs delivered during the next step's GPU time
        self._embed_ready: dict = {}  # pooling slot -> embedding read at its step's commit
        self._next_id = 1
        self._id_lock = threading.Lock()
        self._thread: Optional[threading.Thread] = None
        self._stop = False
        self._err: Optional[BaseException] = None
        self.timings: "deque" = deque(maxlen=1 << 20)  # (ttft_s, tpot_s, output_tokens) per request
        self.stats = {"steps": 0, "tokens": 0, "sampled": 0, "requests": 0, "finished": 0,
                      "embed_requests": 0, "embed_tokens": 0,
                      "busy_s": 0.0, "prefill_tokens": 0, "decode_steps": 0, "graph_replays": 0, "graph_captures": 0,
                      "bucket_tokens": 0, "host_sched_s": 0.0, "host_launch_s": 0.0, "device_wait_s": 0.0,
                      "host_commit_s": 0.0, "host_deliver_s": 0.0}
        self.bucket_hist: Dict[int, list] = {}  # bucket -> [steps, seconds]
        # called on the engine thread right after a step is launched with its token count (the
        # memory batcher co-schedules its index scans with compute-bound steps, memory/batcher.py)
        self._step_listeners: List[Callable[[int], None]] = []
        # custom all-reduce health: its spin-waits give up after ~5 s and set an error word
        # instead of hanging; the word is copied back with every step and checked after the
        # step's synchronize, failing the engine rather than continuing on partial sums
        self._car = getattr(self.tp, "custom", None) if self.tp.size > 1 else None
        # device health words read back with every step (non-blocking, behind the step) and
        # checked after its synchronize: [0] the custom all-reduce's barrier timeout, [1] the
        # weight-streaming GEMM's split-K group-barrier timeout (gemm_stream.hip: a partner
        # workgroup never became resident, so the reduced slabs would be partial)
        self._health_dev = []
        if self._car is not None:
            self._health_dev.append(("custom all-reduce barrier timed out (a TP peer stalled > 5 s): "
                                     "the step's activations are partial", self._car.err))
        if self.on_gpu:
            self._health_dev.append(("weight-streaming GEMM split-K group barrier timed out (a "
                                     "partner workgroup never ran): the step's projections are partial",
                                     ops.stream_workspace(self.device)[2]))
        self._health_host = torch.zeros(max(1, len(self._health_dev)), dtype=torch.int32, pin_memory=pin)
        self._tp_ring = None
        if self.tp.size > 1:
            self._open_tp_ring()
        if self.tp.size > 1:  # ranks reach graph capture together (their init times differ)
            torch.distributed.barrier(group=self.tp.cpu_group)
        # graphs contain the TP collectives, so every rank captures every bucket up front
        if self.use_graphs and (cfg.capture_on_start or self.tp.size > 1):
            self.capture_graphs()

    # ------------------------------------------------------------------ setup
    def _init_views(self):
        L, d = self.L, self._dev_meta
        ms, mb = L["max_seqs"], L["max_blocks"]

        def sl(name, n):
            o = L[name]
            return d[o:o + n]

        self.meta = StepMeta(
            input_ids=sl("input_ids", L["max_tokens"]),
            positions=sl("positions", L["max_tokens"]),
            slots=sl("slots", L["max_tokens"]),
            q_start=sl("q_start", ms), q_len=sl("q_len", ms), ctx_len=sl("ctx_len", ms),
            block_table=sl("block_table", ms * mb).view(ms, mb),
            items=sl("items", 4 * L["max_items"]).view(L["max_items"], 4),
            n_items=sl("n_items", 1),
            att_counters=self._att_counters,
            part_size=sl("part_size", 1),
            logit_rows=sl("logit_rows", ms))
        self._temp = sl("temperature", ms).view(torch.float32)
        self._top_k = sl("top_k", ms)
        self._top_p = sl("top_p", ms).view(torch.float32)
        self._mask_cls = sl("mask_class", ms)
        self._forced = sl("forced", ms)
        self._offsets = sl("offsets", ms)
        self._seeds = sl("seeds", 2 * ms).view(torch.int64)

    def _sync_masks(self) -> bool:
        reg = self.grammar.reg
        if reg.version == self._mask_version:
            return False
        packed = torch.from_numpy(reg.packed())
        self._class_masks[: packed.shape[0]].copy_(packed.to(self.device))
        self._mask_version = reg.version
        return True

    def _items_for_bucket(self, bucket: int, s_b: int) -> int:
        return min(self.L["max_items"], bucket // (2 * self._tpw) + s_b * (self._max_parts + 1) + 4)

    def _meta_for(self, bucket: int, s_b: int, ns: int) -> StepMeta:
        m = self.meta
        n_it = self._items_for_bucket(bucket, s_b)
        return StepMeta(m.input_ids, m.positions, m.slots, m.q_start, m.q_len, m.ctx_len,
                        m.block_table, m.items[:n_it], m.n_items, m.att_counters, m.logit_rows, num_seqs=ns,
                        part_size=m.part_size)

    def _forward_and_sample(self, bucket: int, s_b: int, ns: int, trunc: bool = False, embed: bool = False):
        meta = self._meta_for(bucket, s_b, ns)
        if self._async:  # pending tokens of rows that sampled in the previous step
            ops.patch_pending_ids(meta.input_ids[:bucket], self._sampled_dev)
        logits = self.model.forward(meta, self.kv, bucket, s_b, self._part_o, self._part_ml,
                                    embed=(self._embed_rows, self._embed_pool) if embed else None)
        tau = None
        if trunc:
            # exact top-k / top-p threshold on the full vocabulary; under TP from all-reduced
            # per-shard radix histograms (engine/tp_sampling.py), not an all-gather of the logits
            if self.tp.size == 1:
                tau = ops.topkp_threshold(logits, self.model_cfg.vocab_size, self._temp[:s_b], self._top_k[:s_b],
                                          self._top_p[:s_b], self._mask_cls[:s_b], self._class_masks,
                                          out=self._tau[:s_b])
            else:
                tau = tp_topkp_threshold(logits, self.model.vocab_offset, self.model_cfg.vocab_size,
                                         self._temp[:s_b], self._top_k[:s_b], self._top_p[:s_b],
                                         self._mask_cls[:s_b], self._class_masks, self.tp, out=self._tau[:s_b],
                                         ws=self._tkp_ws)
        if self.tp.size == 1:
            ops.sample(logits, self._temp[:s_b], self._mask_cls[:s_b], self._class_masks,
                       self._seeds[:s_b], self._offsets[:s_b], self._forced[:s_b],
                       out=self._sampled_dev[:s_b], workspace=self._sample_ws, tau=tau)
        else:
            # vocab-parallel: local winners + keys, all-gather, global argmax (identical
            # to the TP=1 token because the Gumbel noise is keyed on the global index)
            ops.sample(logits, self._temp[:s_b], self._mask_cls[:s_b], self._class_masks,
                       self._seeds[:s_b], self._offsets[:s_b], self._forced[:s_b],
                       out=self._sampled_dev[:s_b], workspace=self._sample_ws,
                       vocab_offset=self.model.vocab_offset, out_keys=self._keys_dev[:s_b], tau=tau)
            s4 = (s_b + 3) & ~3  # whole 16-byte vectors for the custom all-gather
            keys = self.tp.all_gather(self._keys_dev[:s4])[:, :s_b]        # [tp, s_b]
            toks = self.tp.all_gather(self._sampled_dev[:s4])[:, :s_b]     # [tp, s_b]
            best = keys.argmax(0, keepdim=True)
            self._sampled_dev[:s_b].copy_(toks.gather(0, best).squeeze(0))

    def _run(self, bucket: int, ns: int, trunc: bool, n_copy: int, embed: bool = False):
        """Replay the (bucket, trunc, embed) graph — capturing it first if needed — or run eagerly."""
        if not self.use_graphs:
            self._forward_and_sample(bucket, self._seq_bucket(bucket), ns, trunc, embed)
            return
        g = self._graphs.get((bucket, trunc, embed))
        if g is None:
            saved = self._dev_meta[:n_copy].clone()
            pool = self._embed_pool.clone()
            samp = self._sampled_dev.clone()  # the previous step's tokens (pipelined mode)
            self.capture_graphs([bucket], trunc=trunc, embed=embed)  # clobbers the device metadata
            self.stats["graph_captures"] += 1  # a first-use capture inside serving (tens of ms)
            self._dev_meta[:n_copy].copy_(saved)
            self._embed_pool.copy_(pool)
            self._sampled_dev.copy_(samp)
            g = self._graphs[(bucket, trunc, embed)]
        g.replay()
        self.stats["graph_replays"] += 1

    def _seq_bucket(self, bucket: int) -> int:
        return min(bucket, self.cfg.max_num_seqs)

    def _dummy_meta(self):
        """A metadata state under which a forward touches no KV and no attention item."""
        L = self.L
        d = torch.zeros(L["total"], dtype=torch.int32)
        d[L["slots"]:L["slots"] + L["max_tokens"]] = -1
        d[L["embed_rows"]:L["embed_rows"] + L["max_tokens"]] = L["max_seqs"]
        self._dev_meta.copy_(d.to(self.device))

    def capture_embed_graphs(self):
        """Capture every bucket's embedding-pooling variant now (before start()), so embedding
        requests never pay a first-use capture (tens of ms each) while serving."""
        if self._thread is not None:
            raise RuntimeError("capture_embed_graphs() runs before start()")
        self.capture_graphs(embed=True)

    def capture_graphs(self, buckets: Optional[Sequence[int]] = None, trunc: bool = False, embed: bool = False):
        """Capture one hipGraph per token bucket (shared memory pool); the top-k/top-p and
        embedding-pooling variants are captured on first use."""
        if not self.use_graphs:
            return
        self._dummy_meta()
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        t0 = time.time()
        for b in sorted(buckets or self.buckets, reverse=True):
            if (b, trunc, embed) in self._graphs:
                continue
            s_b = self._seq_bucket(b)
            st = torch.cuda.Stream(device=self.device)
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st):
                for _ in range(2):
                    self._forward_and_sample(b, s_b, 0, trunc, embed)
            torch.cuda.current_stream().wait_stream(st)
            g = torch.cuda.CUDAGraph(keep_graph=True) if self.cfg.keep_graphs else torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self._graph_pool):
                self._forward_and_sample(b, s_b, 0, trunc, embed)
            if self.cfg.keep_graphs:
                g.instantiate()
            self._graphs[(b, trunc, embed)] = g
        if embed:
            self._embed_pool.zero_()  # the capture's dummy steps pooled into row max_seqs only
        torch.cuda.synchronize()
        log.info("captured %d hipGraphs in %.1fs", len(self._graphs), time.time() - t0)

    # ------------------------------------------------------------------ API
    def new_request_id(self) -> int:
        with self._id_lock:
            rid = self._next_id
            self._next_id += 1
            return rid

    def submit(self, prompt_ids: Sequence[int], callback: Callable[[GenerationOutput], None], *,
               temperature: float = 0.7, max_tokens: int = 256, seed: Optional[int] = None,
               ignore_eos: bool = False, stop_ids: Sequence[int] = (), grammar: Optional[list] = None,
               request_id: Optional[int] = None, top_k: int = 0, top_p: float = 1.0,
               embed: Union[bool, str] = False) -> int:
        """Thread-safe; `callback` runs on the engine thread when the request finishes.

        top_k > 0 / top_p < 1 truncate the (grammar-masked) distribution before
        sampling (exact threshold kernel, csrc/ops/sampling.hip). embed=True (or "mean"): an
        embedding request — the prompt is prefilled in the continuous batch (no prefix-cache
        reuse), nothing is sampled, and the output carries the mean final-norm hidden state.
        embed="last": the final-norm hidden state of the prompt's last token; since a token's
        state depends only on its prefix, such requests reuse cached prefix blocks (shared
        task text across an agent's lookups is computed once)."""
        if self._err is not None:
            raise RuntimeError(f"engine failed: {self._err!r}")
        rid = request_id if request_id is not None else self.new_request_id()
        if seed is None:
            seed = (self.cfg.seed * 0x9E3779B1 + rid * 0x85EBCA77) & 0x7FFFFFFFFFFFFFFF
        req = _Request(rid, list(prompt_ids), float(temperature), int(max_tokens), int(seed),
                       bool(ignore_eos), list(stop_ids), grammar, callback, self._rt.now(),
                       int(top_k or 0), float(1.0 if top_p is None else top_p), bool(embed), embed == "last")
        self._inbox.put(req)
        self._wake.set()
        return rid

    def add_step_listener(self, fn: Callable[[int], None]):
        """fn(tokens) runs on the engine thread right after each step is launched (keep it cheap:
        e.g. loop.call_soon_threadsafe). The kind of step the device is about to run."""
        self._step_listeners = self._step_listeners + [fn]  # copy-on-write: the engine thread iterates

    def remove_step_listener(self, fn: Callable[[int], None]):
        self._step_listeners = [f for f in self._step_listeners if f is not fn]

    def _notify_launch(self, T: int):
        for fn in self._step_listeners:
            try:
                fn(T)
            except Exception:  # noqa: BLE001 -- a listener must not stop the engine
                log.exception("step listener failed")

    def abort(self, rid: int):
        self._aborts.put(rid)
        self._wake.set()

    def generate(self, prompts: Sequence[Sequence[int]], **kw) -> List[GenerationOutput]:
        """Blocking batch generation (drives the loop inline if no thread is running)."""
        results: Dict[int, GenerationOutput] = {}
        done = threading.Event()
        ids = []
        lock = threading.Lock()

        def cb(o: GenerationOutput):
            with lock:
                results[o.request_id] = o
                if len(results) == len(prompts):
                    done.set()

        for p in prompts:
            ids.append(self.submit(p, cb, **kw))
        if self._thread is None:
            while not done.is_set():
                if not self.step():
                    if not self.sched.has_work() and self._inbox.empty():
                        break
        else:
            done.wait()
        if self._err is not None:
            raise RuntimeError(f"engine failed: {self._err!r}")
        return [results[i] for i in ids]

    def embed(self, prompts: Sequence[Sequence[int]], pooling: str = "mean") -> np.ndarray:
        """Final-norm hidden state of each prompt, mean-pooled (pooling="mean") or of its last
        token ("last": reuses cached prefix blocks), [B, hidden] fp32, computed as embedding
        requests inside the continuous batch (the engine's own kernels and graphs, batched
        with whatever else is running). Blocking; thread-safe."""
        if pooling not in ("mean", "last"):
            raise ValueError(f"pooling must be 'mean' or 'last', not {pooling!r}")
        outs = self.generate([list(p) or [0] for p in prompts], embed="last" if pooling == "last" else True,
                             temperature=0.0, max_tokens=1)
        bad = [o.finish_reason for o in outs if o.embedding is None]
        if bad:
            raise RuntimeError(f"embedding requests did not complete: {bad}")
        return np.stack([o.embedding for o in outs]) if outs else np.zeros((0, self.model_cfg.hidden_size), np.float32)

    def prewarm(self, prompt_ids: Sequence[int], timeout: float = 300.0) -> int:
        """Compute and cache the KV of `prompt_ids` (prefix cache) without keeping
        the request; returns the number of prompt tokens. Works with or without
        the engine thread running."""
        if self._thread is None:
            return self.generate([list(prompt_ids)], temperature=0.0, max_tokens=1, ignore_eos=True)[0].prompt_tokens
        done = threading.Event()
        box = {}

        def cb(o):
            box["o"] = o
            done.set()

        self.submit(list(prompt_ids), cb, temperature=0.0, max_tokens=1, ignore_eos=True)
        if not done.wait(timeout):
            raise TimeoutError("prewarm did not finish")
        return box["o"].prompt_tokens

    def start(self):
        if self._thread is not None:
            return
        sw = self.cfg.gil_switch_interval
        if sw is None and os.environ.get("PILOTTAI_GIL_SWITCH_S"):
            sw = float(os.environ["PILOTTAI_GIL_SWITCH_S"])
        if sw is not None and sw > 0:
            sys.setswitchinterval(sw)
        self._stop = False
        if self.cfg.freeze_heap:
            # the model, graphs and tokenizer are in place: keep them out of every later GC
            # pass (a full collection otherwise stalls the engine thread for tens of ms)
            from pilottai_amd.utils.gc_tune import freeze_heap

            self._froze = freeze_heap() > 0
        self._thread = threading.Thread(target=self._loop, name="pilottai-engine", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop = True
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None
        if getattr(self, "_froze", False):  # give the frozen heap back to the collector
            import gc

            gc.unfreeze()
            self._froze = False
        self.release_followers()

    # ------------------------------------------------------------------ TP
    def _open_tp_ring(self):
        """The per-step TP header travels through a shared-memory ring (csrc/runtime/shm_ring.cpp;
        SURVEY §5: shared-memory rings, not sockets, for the node-local control hop): the
        driver publishes, every follower polls its own read position. PILOTTAI_TP_HEADER=gloo
        (or a node without POSIX shared memory) keeps the gloo broadcast."""
        if os.environ.get("PILOTTAI_TP_HEADER", "shm") == "gloo":
            return
        box = [f"pilottai_tp_{os.getpid()}_{self.tp.root}_{os.urandom(4).hex()}" if self.is_driver else None]
        torch.distributed.broadcast_object_list(box, src=self.tp.root, group=self.tp.cpu_group)
        # Symmetric two-phase handshake: every rank reaches the same two collectives whatever
        # fails where (a driver-side create failure must not leave the followers in a barrier
        # that the driver skipped). Phase 1: the driver creates, all ranks agree on the status;
        # phase 2: the followers attach, all ranks agree again. Any failure -> gloo everywhere.
        created = self._tp_ring_phase(lambda rt: self._set_tp_ring(rt.ShmRing(box[0], 9, 64, self.tp.size - 1, True))
                                      if self.is_driver else None, "create")
        attached = created and self._tp_ring_phase(
            lambda rt: self._set_tp_ring(rt.ShmRing(box[0], 9, 64, self.tp.size - 1, False, 120.0))
            if not self.is_driver else None, "attach")
        if not attached:
            self._tp_ring = None

    def _set_tp_ring(self, ring):
        self._tp_ring = ring

    def _tp_ring_phase(self, fn, what: str) -> bool:
        """Run fn(_runtime) on this rank, then all-reduce the failure flag over the TP group:
        True iff the phase succeeded on every rank."""
        bad = torch.zeros(1, dtype=torch.int32)
        try:
            from pilottai_amd import _runtime

            if os.environ.get("PILOTTAI_TP_RING_FAIL") == f"{what}:{self.tp.rank}":  # fault injection (tests)
                raise RuntimeError(f"injected TP ring {what} failure")
            fn(_runtime)
        except Exception as e:  # noqa: BLE001 — fall back to the gloo broadcast on every rank
            log.warning("TP header ring %s failed on rank %d (%s): using the gloo broadcast", what, self.tp.rank, e)
            bad[0] = 1
        torch.distributed.all_reduce(bad, group=self.tp.cpu_group)
        return int(bad[0]) == 0

    def _tp_send(self, op: int, *vals: int):
        h = self._tp_header
        h.zero_()
        h[0] = op
        for i, v in enumerate(vals):
            h[1 + i] = int(v)
        if self._tp_ring is not None:
            if not self._tp_ring.put(h.tolist(), 600.0):
                raise RuntimeError("TP follower stopped reading step headers (ring full for 600 s)")
        else:
            self.tp.broadcast(h, cpu=True)

    def _tp_recv(self):
        if self._tp_ring is not None:
            rec = self._tp_ring.get(self.tp.rank - 1, 3600.0)
            if rec is None:
                raise RuntimeError("no TP step header from the driver for an hour")
            return rec
        self.tp.broadcast(self._tp_header, cpu=True)
        return self._tp_header.tolist()

    def release_followers(self):
        """Driver: tell the follower ranks to leave `follow()` (idempotent)."""
        if self.tp.size > 1 and self.is_driver and not self._tp_closed:
            self._tp_closed = True
            self._tp_send(_OP_STOP)

    def follow(self) -> int:
        """Follower ranks (TP rank > 0): mirror the driver's steps until it stops.

        Returns the number of steps executed."""
        if self.is_driver:
            raise RuntimeError("follow() is for TP ranks > 0")
        if self.on_gpu:
            torch.cuda.set_device(self.device)
        n = 0
        with torch.inference_mode():
            while True:
                op, T, ns, nsamp, bucket, masks_changed, n_copy, trunc, embed = (int(v) for v in self._tp_recv())
                if op == _OP_STOP:
                    break
                if masks_changed:
                    self.tp.broadcast(self._class_masks)
                self.tp.broadcast(self._dev_meta[:n_copy])
                self._run(bucket, ns, bool(trunc), n_copy, bool(embed))
                self._health_fetch()
                if self.on_gpu:
                    torch.cuda.current_stream().synchronize()
                self._health_check()
                n += 1
        self.stats["steps"] += n
        return n

    def _health_fetch(self):
        for i, (_, w) in enumerate(self._health_dev):
            self._health_host[i:i + 1].copy_(w[:1], non_blocking=True)

    def _health_check(self):
        """Fail the engine (rather than continue on partial sums) if a device health word is
        set; call after the step's synchronize."""
        for i, (what, _) in enumerate(self._health_dev):
            if int(self._health_host[i]) != 0:
                raise RuntimeError(f"{what}; engine stopped")

    @property
    def failed(self) -> Optional[BaseException]:
        return self._err

    # ------------------------------------------------------------------ loop
    def _drain_inbox(self):
        while True:
            try:
                req: _Request = self._inbox.get_nowait()
            except queue.Empty:
                break
            self._reqs[req.rid] = req
            self.sched.add_request(req.rid, req.prompt_ids, req.temperature, req.max_tokens, req.seed,
                                   req.ignore_eos, req.stop_ids, req.grammar, req.top_k, req.top_p, req.embed,
                                   req.embed_last)
            self.stats["requests"] += 1
        while True:
            try:
                rid = self._aborts.get_nowait()
            except queue.Empty:
                break
            self.sched.abort(rid)
        for o in self.sched.drain_aborted():
            self._deliver(o)

    def _deliver(self, o):
        rid, toks, reason, plen, cached, nsamp, nforced, t_first, t_fin, eslot = o
        emb = None
        if eslot >= 0 and eslot in self._embed_ready:  # read back when its step committed
            emb = self._embed_ready.pop(eslot)
        elif eslot >= 0:  # (aborted / not yet read) the request's pooling row: read and clear it
            if reason == 3:
                emb = (self._embed_pool[eslot] / self._pool_div(rid, plen)).cpu().numpy()
            self._embed_pool[eslot].zero_()
        if reason == 3:
            self.stats["embed_requests"] += 1
            self.stats["embed_tokens"] += plen - cached
            self.stats["embed_cached_tokens"] = self.stats.get("embed_cached_tokens", 0) + cached
        req = self._reqs.pop(rid, None)
        self.stats["finished"] += 1
        if req is None:
            return
        out = GenerationOutput(rid, list(toks), _REASONS.get(reason, "stop"), plen, cached, len(toks),
                               nsamp, nforced, req.t_arrival, t_first, t_fin, self.tok, emb)
        # per-request timings: TTFT = arrival -> first token, TPOT = later tokens' mean gap
        if t_first > 0:
            n_out = max(1, len(toks))
            self.timings.append((out.ttft, (t_fin - t_first) / max(1, n_out - 1), n_out))
        try:
            req.callback(out)
        except Exception:  # noqa: BLE001 — a bad callback must not kill the engine
            log.exception("completion callback failed")

    def step(self) -> bool:
        """Run one engine step. Returns False when there was nothing to run."""
        if self._async:
            return self._step_pipelined()
        self._drain_inbox()
        if not self.sched.has_work():
            self._flush_deliveries()
            return False
        L = self.L
        t0 = time.perf_counter()
        with trace_range("engine.schedule"):
            T = self.sched.schedule(self._host_ptr)
        t_sched = time.perf_counter()
        if T == 0:
            self._flush_deliveries()
            if self.sched.num_running == 0 and self.sched.num_waiting > 0:
                raise RuntimeError("KV cache too small for the head request")
            return False
        c = self._host_np[L["counts"]:L["counts"] + 8]
        ns, nsamp, trunc, embed = int(c[1]), int(c[2]), int(c[6]) > 0, int(c[7]) > 0
        bucket = next(b for b in self.buckets if b >= T)
        s_b = self._seq_bucket(bucket)
        masks_changed = self._sync_masks()
        n_copy = L["embed_rows"] + bucket if embed else L["block_table"] + ns * L["max_blocks"]
        resets = self.sched.take_embed_resets()
        if resets:  # preempted embedding requests restart from token 0
            self._embed_pool[torch.tensor(resets, dtype=torch.long, device=self.device)] = 0.0
        if self.on_gpu:
            self._dev_meta[:n_copy].copy_(self._host_meta[:n_copy], non_blocking=True)
        if self.tp.size > 1:
            self._tp_send(_OP_STEP, T, ns, nsamp, bucket, int(masks_changed), n_copy, int(trunc), int(embed))
            if masks_changed:
                self.tp.broadcast(self._class_masks)
            self.tp.broadcast(self._dev_meta[:n_copy])
        with torch.inference_mode(), trace_range("engine.forward"):
            self._run(bucket, ns, trunc, n_copy, embed)
        if self._step_listeners:
            self._notify_launch(T)
        if nsamp:
            self._sampled_host[:nsamp].copy_(self._sampled_dev[:nsamp], non_blocking=self.on_gpu)
        self._health_fetch()
        t_launch = time.perf_counter()
        # the previous step's finished requests are handed to their callers while this step
        # runs on the GPU (host/device overlap): delivery needs nothing from it
        self._flush_deliveries()
        t_flush = time.perf_counter()
        if self.on_gpu:
            torch.cuda.current_stream().synchronize()
        self._health_check()
        t_sync = time.perf_counter()
        with trace_range("engine.commit"):
            outs = self.sched.commit(self._sampled_host.data_ptr(), nsamp)
        if embed:
            self._read_embeddings(outs)
        st = self.stats
        # host-side phases: schedule, metadata copy + launch, device wait, commit
        st["host_sched_s"] += t_sched - t0
        st["host_launch_s"] += t_launch - t_sched
        st["device_wait_s"] += t_sync - t_launch
        st["steps"] += 1
        st["tokens"] += T
        st["bucket_tokens"] += bucket
        st["sampled"] += nsamp
        dt = time.perf_counter() - t0
        st["busy_s"] += dt
        bh = self.bucket_hist.setdefault(bucket, [0, 0.0])
        bh[0] += 1
        bh[1] += dt
        st["host_commit_s"] += time.perf_counter() - t_sync
        st["host_deliver_s"] += t_flush - t_launch  # overlapped with the device
        self._pending_out.extend(outs)
        if not self.sched.has_work():
            self._flush_deliveries()  # nothing to overlap with: deliver now
        return True

    # ------------------------------------------------------------- pipelined steps
    def _step_pipelined(self) -> bool:
        """One turn of the pipelined loop: launch the next step if fewer than two are in
        flight, then (with two in flight, or nothing new to launch) wait for the oldest and
        commit it. In steady state step N+1 is scheduled, copied and launched while step N
        runs on the device, so the device never waits for the host's schedule / launch /
        commit (0.5-0.6 ms per step in the serial loop, BENCH_r02 step_phase_ms)."""
        self._drain_inbox()
        launched = False
        if len(self._inflight) < 2 and self.sched.has_work():
            launched = self._launch_next()
        if self._inflight and (len(self._inflight) == 2 or not launched):
            self._complete(self._inflight.popleft())
            return True
        if not launched:
            self._flush_deliveries()
        return launched

    def _launch_next(self) -> bool:
        L = self.L
        slot = self._slot
        hm = self._host_metas[slot]
        t0 = time.perf_counter()
        with trace_range("engine.schedule"):
            T = self.sched.schedule(hm.data_ptr())
        t_sched = time.perf_counter()
        if T == 0:
            if not self._inflight and self.sched.num_running == 0 and self.sched.num_waiting > 0:
                raise RuntimeError("KV cache too small for the head request")
            return False
        c = hm.numpy()[L["counts"]:L["counts"] + 8]
        ns, nsamp, trunc, embed = int(c[1]), int(c[2]), int(c[6]) > 0, int(c[7]) > 0
        bucket = next(b for b in self.buckets if b >= T)
        self._sync_masks()
        n_copy = L["embed_rows"] + bucket if embed else L["block_table"] + ns * L["max_blocks"]
        resets = self.sched.take_embed_resets()
        if resets:
            self._embed_pool[torch.tensor(resets, dtype=torch.long, device=self.device)] = 0.0
        self._dev_meta[:n_copy].copy_(hm[:n_copy], non_blocking=self.on_gpu)
        with torch.inference_mode(), trace_range("engine.forward"):
            self._run(bucket, ns, trunc, n_copy, embed)
        if self._step_listeners:
            self._notify_launch(T)
        if nsamp:
            self._sampled_hosts[slot][:nsamp].copy_(self._sampled_dev[:nsamp], non_blocking=self.on_gpu)
        if embed:
            self._embed_hosts[slot].copy_(self._embed_pool, non_blocking=self.on_gpu)
        self._health_fetch()
        ev = None
        if self.on_gpu:
            ev = torch.cuda.Event()
            ev.record()
        t_launch = time.perf_counter()
        self._inflight.append((slot, T, bucket, nsamp, embed, ev, t0))
        self._slot = (slot + 1) % len(self._host_metas)
        st = self.stats
        st["host_sched_s"] += t_sched - t0
        st["host_launch_s"] += t_launch - t_sched
        self._flush_deliveries()  # the previous step's outputs, while this one is queued
        st["host_deliver_s"] += time.perf_counter() - t_launch
        return True

    def _complete(self, rec):
        slot, T, bucket, nsamp, embed, ev, t0 = rec
        t_w = time.perf_counter()
        if ev is not None:
            ev.synchronize()
        self._health_check()
        t_sync = time.perf_counter()
        with trace_range("engine.commit"):
            outs = self.sched.commit(self._sampled_hosts[slot].data_ptr(), nsamp)
        if embed:
            self._read_embeddings(outs, self._embed_hosts[slot])
        st = self.stats
        st["device_wait_s"] += t_sync - t_w
        st["steps"] += 1
        st["tokens"] += T
        st["bucket_tokens"] += bucket
        st["sampled"] += nsamp
        # device time attributable to this step: from its launch (or the previous step's
        # completion, whichever is later) to its completion
        dt = t_sync - max(t0, self._last_done)
        self._last_done = t_sync
        st["busy_s"] += dt
        bh = self.bucket_hist.setdefault(bucket, [0, 0.0])
        bh[0] += 1
        bh[1] += dt
        st["host_commit_s"] += time.perf_counter() - t_sync
        self._pending_out.extend(outs)
        if not self._inflight and not self.sched.has_work():
            self._flush_deliveries()

    def _read_embeddings(self, outs, host: Optional[torch.Tensor] = None):
        """Pooled rows of the embedding requests this step finished. Serial loop: read from
        the device while it is idle (step synchronised). Pipelined loop: from `host`, the
        pinned snapshot taken behind this step (the next step is already queued, so a device
        read would wait for it too). Delivery runs during the NEXT step either way."""
        done = [(o[9], self._pool_div(o[0], o[3])) for o in outs if o[9] >= 0 and o[2] == 3]
        if not done:
            return
        slots = [e for e, _ in done]
        idx = torch.tensor(slots, dtype=torch.long, device=self.device)
        rows = host.numpy()[slots] if host is not None else self._embed_pool.index_select(0, idx).cpu().numpy()
        # stream-ordered: a finished request's row takes no more tokens in the queued step
        self._embed_pool.index_fill_(0, idx, 0.0)
        for (e, plen), r in zip(done, rows):
            self._embed_ready[e] = r / plen

    def _pool_div(self, rid: int, plen: int) -> int:
        """Tokens pooled into an embedding request's row: its prompt (mean), or 1 (last)."""
        req = self._reqs.get(rid)
        return 1 if (req is not None and req.embed_last) else max(1, plen)

    def _flush_deliveries(self):
        if self._pending_out:
            outs, self._pending_out = self._pending_out, []
            for o in outs:
                self._deliver(o)

    def _loop(self):
        if self.on_gpu:
            torch.cuda.set_device(self.device)
        try:
            while not self._stop:
                if not self.step():
                    self._wake.wait(0.01)
                    self._wake.clear()
        except BaseException as e:  # noqa: BLE001
            self._err = e
            log.exception("engine loop crashed")
            # requests that already finished (held for overlapped delivery) get their outputs
            try:
                self._flush_deliveries()
            except Exception:  # noqa: BLE001
                log.exception("delivery after the crash failed")
            # fail every other pending request loudly
            for rid in list(self._reqs):
                req = self._reqs.pop(rid)
                try:
                    req.callback(GenerationOutput(rid, [], "error", len(req.prompt_ids), 0, 0, 0, 0,
                                                  req.t_arrival, -1.0, self._rt.now(), self.tok))
                except Exception:  # noqa: BLE001
                    pass

    # ------------------------------------------------------------------ info
    def latency_summary(self, since: int = 0) -> dict:
        """p50/p99 TTFT and TPOT (ms) over requests finished after index `since`."""
        tm = list(self.timings)[since:]
        if not tm:
            return {}
        ttft = sorted(t[0] for t in tm)
        tpot = sorted(t[1] for t in tm if t[2] > 1)
        pick = lambda v, q: 1000 * v[min(len(v) - 1, int(q * len(v)))] if v else None  # noqa: E731
        return {"requests": len(tm), "ttft_p50_ms": pick(ttft, 0.5), "ttft_p99_ms": pick(ttft, 0.99),
                "tpot_p50_ms": pick(tpot, 0.5), "tpot_p99_ms": pick(tpot, 0.99)}

    def metrics(self) -> dict:
        s = self.sched
        st = dict(self.stats)
        st.update({
            "running": s.num_running, "waiting": s.num_waiting, "free_kv_blocks": s.num_free_blocks,
            "total_kv_blocks": self.num_kv_blocks, "cached_kv_blocks": s.num_cached_blocks,
            "prompt_tokens": s.total_prompt_tokens, "prefix_cache_hit_tokens": s.total_cached_tokens,
            "preemptions": s.total_preemptions, "graphs": len(self._graphs), "aligned_steps": s.aligned_steps,
            "prefix_defers": s.prefix_defers,
            "spec_rows": s.spec_rows, "spec_voided": s.spec_voided,
            "kv_cache_gb": self.kv.k.numel() * 2 * 2 / 2**30,
            "weights_gb": self.model.weight_bytes() / 2**30,
        })
        if self.on_gpu:
            st["hbm_used_gb"] = torch.cuda.memory_allocated(self.device) / 2**30
        return st
