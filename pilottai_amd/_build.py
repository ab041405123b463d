"""In-tree builder for the native parts of pilottai_amd.

Two shared objects are produced next to the Python sources so they travel with
the repository snapshot to the GPU box:

* ``pilottai_amd/_C.so``       — CDNA4 HIP kernels (csrc/ops/*.hip, gfx950 only)
                                  + torch/pybind11 bindings (csrc/ops/bindings.cpp)
* ``pilottai_amd/_runtime.so`` — C++ serving runtime: paged-KV block manager,
                                  prefix cache, continuous-batching scheduler,
                                  grammar FSM + tokenizer (csrc/runtime/*.cpp),
                                  pybind11 bindings, no GPU code.

hipcc is driven directly (no hipify, no torch JIT cache): each translation unit
is compiled to an object in ``build/`` and re-linked only when a source or
header changed. Usage: ``python -m pilottai_amd._build`` or ``build_all()``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "pilottai_amd"
CSRC = ROOT / "csrc"
BUILD = ROOT / "build"
ARCH = os.environ.get("PILOTTAI_GPU_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# Per-file code-generation flags. gemm_mid.hip: MFMA accumulators in the VGPR form; with
# the AGPR form hipcc shuffles them through v_accvgpr moves in the software-pipelined loop.
FILE_FLAGS = {"gemm_mid.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"],
              "gemm_stream.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _torch_paths():
    from torch.utils import cpp_extension as ce

    return ce.include_paths(), ce.library_paths()


def _py_include() -> str:
    return sysconfig.get_paths()["include"]


def _pybind_include() -> str:
    import pybind11

    return pybind11.get_include()


def _newest(paths) -> float:
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _compile_many(jobs, workers: int):
    todo = [(src, obj, cmd) for src, obj, cmd, deps in jobs
            if not os.path.exists(obj) or os.path.getmtime(obj) < _newest([src] + deps)]
    if not todo:
        return 0
    with cf.ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        futs = [ex.submit(_run, cmd) for _, _, cmd in todo]
        for f in futs:
            f.result()
    return len(todo)


def build_ops(verbose: bool = False, workers: int | None = None) -> Path:
    """Compile csrc/ops into pilottai_amd/_C.so (gfx950 code objects)."""
    incs, libdirs = _torch_paths()
    out = PKG / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))
    BUILD.mkdir(exist_ok=True)
    headers = glob.glob(str(CSRC / "ops" / "*.h"))
    jobs = []
    objs = []
    for src in sorted(glob.glob(str(CSRC / "ops" / "*.hip"))):
        obj = str(BUILD / (Path(src).stem + ".hip.o"))
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src,
               "-o", obj, "-ffast-math", "-fno-gpu-rdc", "-Wno-unused-result",
               *FILE_FLAGS.get(Path(src).name, [])]
        jobs.append((src, obj, cmd, headers))
        objs.append(obj)
    bsrc = str(CSRC / "ops" / "bindings.cpp")
    bobj = str(BUILD / "ops_bindings.o")
    defs = ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_C",
            "-DTORCH_API_INCLUDE_EXTENSION_H", "-D_GLIBCXX_USE_CXX11_ABI=1"]
    bcmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-c", bsrc, "-o", bobj, *defs,
            "-I/opt/rocm/include", f"-I{_py_include()}"] + [f"-I{i}" for i in incs]
    jobs.append((bsrc, bobj, bcmd, []))
    objs.append(bobj)
    n = _compile_many(jobs, workers or min(8, os.cpu_count() or 4))
    if n or not out.exists() or out.stat().st_mtime < _newest(objs):
        link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(out), *objs]
        for d in libdirs:
            link += [f"-L{d}", f"-Wl,-rpath,{d}"]
        link += ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
                 "-ltorch_python", "-lamdhip64"]
        _run(link)
        if verbose:
            print(f"[pilottai_amd] linked {out}")
    return out


def build_runtime(verbose: bool = False, workers: int | None = None) -> Path:
    """Compile csrc/runtime (pure C++17, no torch) into pilottai_amd/_runtime.so."""
    out = PKG / ("_runtime" + sysconfig.get_config_var("EXT_SUFFIX"))
    BUILD.mkdir(exist_ok=True)
    srcs = sorted(glob.glob(str(CSRC / "runtime" / "*.cpp")))
    headers = glob.glob(str(CSRC / "runtime" / "*.h"))
    jobs, objs = [], []
    flags = os.environ.get("PILOTTAI_RUNTIME_CXXFLAGS", "-O3").split()
    for src in srcs:
        obj = str(BUILD / (Path(src).stem + ".rt.o"))
        cmd = ["g++", *flags, "-std=c++17", "-fPIC", "-Wall", "-c", src, "-o", obj,
               f"-I{_py_include()}", f"-I{_pybind_include()}", f"-I{CSRC / 'runtime'}"]
        jobs.append((src, obj, cmd, headers))
        objs.append(obj)
    n = _compile_many(jobs, workers or min(8, os.cpu_count() or 4))
    if objs and (n or not out.exists() or out.stat().st_mtime < _newest(objs)):
        _run(["g++", "-shared", "-fPIC", *flags, "-o", str(out), *objs, "-lpthread"])
        if verbose:
            print(f"[pilottai_amd] linked {out}")
    return out


def build_all(verbose: bool = False) -> None:
    build_runtime(verbose)
    build_ops(verbose)


if __name__ == "__main__":
    build_all(verbose=True)
    sys.exit(0)
