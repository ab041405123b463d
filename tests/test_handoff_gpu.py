"""In-launch hand-offs under stress (common.h handoff_last): every split-K / partition merge
configuration the engine uses, plus round 2's failing one, with FRESH random inputs each
repetition, the slab workspaces and the outputs NaN-poisoned before every launch and a
side-stream GEMM running beside every other repetition. Any stale or early slab read shows
up as a mismatch against the same kernel without a hand-off (tools/splitk_check.py runs the
same cases for thousands of repetitions: profiles/r3_splitk_handoff.md)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_handoff_survives_poisoned_varied_input_stress(gpu, tmp_path):
    out = tmp_path / "splitk.jsonl"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "splitk_check.py"), "--reps", "150",
                        "--out", str(out)], capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    import json

    recs = [json.loads(line) for line in out.read_text().splitlines()]
    assert len(recs) >= 20, recs
    errors = [r for r in recs if "error" in r]
    bad = [r for r in recs if r.get("bad_runs")]
    assert not errors and not bad, (errors, bad)
