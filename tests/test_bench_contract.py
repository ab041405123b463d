"""bench.py driver contract over 2 ranks (gloo, tiny model on CPU).

The driver launches `torch.distributed.run --nproc-per-node N ... bench.py --gpus N --steps K
--warmup W` and reads ONE JSON line from rank 0. This runs that exact launch shape with
world_size 2 on CPU and checks the line: one line only, the BASELINE metric, agent-DP over
both ranks, the timed-step count, and tasks from both ranks' shards.
"""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


import pytest


@pytest.mark.parametrize("n,launcher,rehearsal", [(2, True, None), (8, True, None), (2, False, None),
                                                  (2, True, "share-gpu"), (2, True, "hybrid")])
def test_bench_multi_rank_json_contract(tmp_path, n, launcher, rehearsal):
    """n ranks under the driver's torchrun launch shape; (2, False): `bench.py --gpus 2`
    without a launcher must start the 2 ranks itself, never silently run one. The scale-run
    evidence fields: n_gpus counts the physical devices the ranks used (0 on
    CPU), the rehearsal flags are named, and the process group's backend / world size and every
    rank's device are reported."""
    env = dict(os.environ, PILOTTAI_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--cpu", "--steps", "1", "--warmup", "1",
            "--workers", str(n), "--doc-words", "20"]
    args += {"share-gpu": ["--share-gpu"], "hybrid": ["--hybrid-latency", "0.01"]}.get(rehearsal, [])
    cmd = ([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
            "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] if launcher else [sys.executable]) + args
    p = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    baseline = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    assert d["metric"] == baseline["metric"]
    assert d["steps"] == 1 and d["warmup"] == 1
    assert d["config"]["parallelism"] == f"agent-dp{n}"
    assert d["config"]["workers"] == n
    assert d["config"]["managers"] == 1  # ONE manager Serve over the node-wide pool
    assert d["tasks"] >= n  # one worker per rank, each completes >= 1 task per timed step
    assert len(d["llm_calls_per_rank"]) == n
    if rehearsal != "hybrid":  # (hybrid: the CPU tiny-model rank 0 is slower than the schema ranks)
        assert all(c > 0 for c in d["llm_calls_per_rank"])
    assert d["value"] > 0 and d["ms_per_step"] > 0
    for k in ("unit", "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 0 and d["physical_devices"] == []  # CPU ranks: no GPU used
    assert d["rehearsal"] == rehearsal
    assert d["dist_backend"] == "gloo" and d["world_size"] == n
    assert d["devices"] == ["cpu"] * n


def test_bench_device_identity_counts_physical_cards():
    """n_gpus is the number of DISTINCT physical cards over the ranks (unit check of the
    identity helper on fake device properties)."""
    import importlib.util
    import types

    import torch

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench._device_identity(torch.device("cpu")) == {"device": "cpu", "physical": None}
    props = types.SimpleNamespace(pci_domain_id=0, pci_bus_id=0x75, pci_device_id=0, name="MI355X", uuid="u")
    orig = torch.cuda.get_device_properties
    try:
        torch.cuda.get_device_properties = lambda i: props
        ident = bench._device_identity(torch.device("cuda", 3))
    finally:
        torch.cuda.get_device_properties = orig
    assert ident["device"] == "cuda:3" and ident["physical"] == "pci:0000:75:00"


def test_bench_node_memory_is_one_sharded_store(tmp_path):
    """in node mode `--memory-rows R` is ONE node-wide store -- R rows in
    total, sharded over the ranks (not R per rank) -- and every agent step's lookups go through
    it (2 gloo ranks, tiny model on CPU)."""
    env = dict(os.environ, PILOTTAI_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    R = 20000
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--cpu", "--steps", "1", "--warmup", "1",
           "--workers", "2", "--doc-words", "20", "--memory-rows", str(R)]
    p = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-3000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    m = d["memory"]
    assert m["store"] == "node-sharded"
    per = m["rows_per_rank"]
    assert len(per) == 2 and R <= sum(per) == m["rows_total"] < R + 1000
    assert all(R // 2 <= r < R // 2 + 1000 for r in per)  # a shard each, plus write-backs
    assert m["lookups"] > 0 and m["node_rounds"] > 0
    # the agents' write-backs reach the node store (none failed), and
    # lookups return rows held by the other rank's shard
    assert m["stores"] > 0 and m["store_failures"] == 0 and m["lookup_failures"] == 0
    assert m["node_hits"] > 0 and m["node_remote_hits"] > 0


def test_bench_agent_dp_over_tp_groups(tmp_path):
    """`--gpus 4 --tp 2` runs 2 agent-DP replicas, each a TP=2 engine (its
    TP rank 1 follows the driver's steps); the node plane and the clients see 2 replicas, the
    JSON line names the layout, and every rank's device is reported (4 gloo ranks on CPU)."""
    env = dict(os.environ, PILOTTAI_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "4", "--tp", "2", "--cpu", "--steps", "1", "--warmup", "1",
           "--workers", "4", "--doc-words", "20"]
    p = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["config"]["parallelism"] == "agent-dp2-tp2"
    assert d["config"]["managers"] == 1 and d["tasks"] >= 4
    assert len(d["llm_calls_per_rank"]) == 2 and all(c > 0 for c in d["llm_calls_per_rank"])
    assert d["world_size"] == 4 and d["devices"] == ["cpu"] * 4
    st = d["tp_selftest"]  # the start-up all-reduce round trip of the TP groups
    assert st["ok"] and st["tp"] == 2 and st["us_64x4096"] > 0 and st["us_2048x4096"] > 0
