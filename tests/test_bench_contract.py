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


@pytest.mark.parametrize("n,launcher", [(2, True), (8, True), (2, False)])
def test_bench_multi_rank_json_contract(tmp_path, n, launcher):
    """n ranks under the driver's torchrun launch shape; (2, False): `bench.py --gpus 2`
    without a launcher must start the 2 ranks itself, never silently run one."""
    env = dict(os.environ, PILOTTAI_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    args = [os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--cpu", "--steps", "1", "--warmup", "1",
            "--workers", str(n), "--doc-words", "20"]
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
    assert len(d["llm_calls_per_rank"]) == n and all(c > 0 for c in d["llm_calls_per_rank"])
    assert d["value"] > 0 and d["ms_per_step"] > 0
    for k in ("unit", "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d
