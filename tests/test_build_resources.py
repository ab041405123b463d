"""Static resource checks of the hand-written kernels (CPU tier: hipcc cross-compiles).

The mid-size GEMM's variant 2 loads its weight ring with untracked inline-asm loads
(csrc/ops/gemm_mid.hip gload16): a register spill between such a load and its counted
wait would store a stale register, so no instantiated kernel may use scratch.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_mid_gemm_kernels_use_no_scratch(tmp_path):
    out = tmp_path / "mid.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-S", "--cuda-device-only",
                    "-ffast-math", "-mllvm", "-amdgpu-mfma-vgpr-form", os.path.join(ROOT, "csrc", "ops", "gemm_mid.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    text = out.read_text()
    sizes = re.findall(r"\.set (_ZN2pa3mid\w+)\.private_seg_size, (\d+)", text)
    assert sizes, "no mid GEMM kernels found in the assembly"
    spilling = [name for name, n in sizes if int(n) > 0]
    assert not spilling, f"kernels with scratch: {spilling}"
    shutil.rmtree(tmp_path, ignore_errors=True)
