"""Per-shape hipBLASLt/rocBLAS solution overrides for the library GEMMs.

tools/tune_gemms.py times every registered solution (PyTorch TunableOp) for each
projection shape at every engine token bucket; the shipped file keeps only the
shapes where the tuned solution beat hipBLASLt's default heuristic by >= 5 %
in cache-warm timing (e.g. down_proj at M=1600: 328 -> 165 us). All other shapes
keep the default. The file is validated by TunableOp against the running
PyTorch / HIP / hipBLASLt / rocBLAS versions and gfx arch; on mismatch it is
ignored.
"""
from __future__ import annotations

import logging
import os
import tempfile

import torch

log = logging.getLogger("pilottai_amd.engine")

TUNED_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuned")
_loaded = set()


def tuned_file(model: str, tp: int) -> str:
    return os.path.join(TUNED_DIR, f"gemm_{model}_tp{tp}.csv")


def load_tuned_gemms(model: str, tp: int = 1) -> bool:
    """Enable TunableOp in replay-only mode with the shipped results for `model`."""
    path = tuned_file(model, tp)
    if not torch.cuda.is_available() or not os.path.exists(path) or os.environ.get("PILOTTAI_NO_TUNED_GEMM"):
        return False
    if path in _loaded:
        return True
    tun = torch.cuda.tunable
    try:
        tun.enable(True)
        tun.tuning_enable(False)
        # results written at exit go to a scratch file, never over the shipped one
        tun.set_filename(os.path.join(tempfile.gettempdir(), f"pilottai_tunableop_{os.getpid()}.csv"))
        ok = tun.read_file(path)
    except Exception as e:  # noqa: BLE001 — tuning is an optimisation only
        log.warning("could not load tuned GEMMs from %s: %s", path, e)
        return False
    if ok:
        _loaded.add(path)
        log.info("loaded tuned GEMM solutions from %s", path)
    return bool(ok)
