"""The native serving runtime under AddressSanitizer + UndefinedBehaviorSanitizer
(the reference has no race/memory checking at all).

Builds csrc/runtime/tests/stress_runtime.cpp together with the runtime sources
(scheduler with preemption + prefix cache + grammar jump-forward + aborts, block
manager fuzz, tokenizer round trips) with -fsanitize=address,undefined and runs it;
any sanitizer report or invariant violation fails the test. CPU tier.
"""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "csrc", "runtime")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_stress_under_asan_ubsan():
    srcs = [os.path.join(RT, "tests", "stress_runtime.cpp")] + [
        os.path.join(RT, f) for f in ("scheduler.cpp", "block_manager.cpp", "grammar.cpp", "tokenizer.cpp")]
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "stress_runtime")
        cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
               "-fno-sanitize-recover=all", f"-I{RT}", *srcs, "-o", exe]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        if r.returncode != 0 and "asan" in (r.stderr or "").lower():
            pytest.skip("toolchain has no AddressSanitizer runtime")
        assert r.returncode == 0, r.stderr[-4000:]
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
        r = subprocess.run([exe, "4"], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
        assert "runtime stress: ok" in r.stdout
        assert r.stdout.count("long-context items") == 4  # seeds 1-2 x GQA groups 4 and 8
        assert "preemptions" in r.stdout and " 0 preemptions" not in r.stdout
