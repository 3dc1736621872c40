"""Build the in-tree native extension ``gsc_amd/_native*.so`` with hipcc for gfx950.

Every ``.hip``/``.cpp`` under ``csrc/`` is compiled to an object (in parallel, skipped when
up to date) and linked into one shared library that contains both the host code (CPU simulator
path, launchers, pybind11 bindings) and the gfx950 code objects.  No torch headers are used:
kernels take raw device pointers and the current HIP stream, which keeps builds fast.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("GSC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> str:
    return os.path.join(ROOT, "gsc_amd", "_native" + sysconfig.get_config_var("EXT_SUFFIX"))


def _includes():
    import pybind11
    return ["-I" + CSRC, "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _flags(src: str):
    f = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result", "-Wno-unused-command-line-argument"]
    if os.sep + "sim" + os.sep in src:
        f.append("-ffp-contract=off")  # bit-exact float semantics vs the Python oracle
    return f


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True)
                  + glob.glob(os.path.join(CSRC, "**", "*.cpp"), recursive=True))


def _headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _obj(src: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    return os.path.join(BUILD, rel + ".o")


def _compile(src: str, newest_header: float) -> str:
    obj = _obj(src)
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), newest_header):
        return obj
    cmd = [HIPCC, "-c", src, "-o", obj] + _flags(src) + _includes()
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose: bool = True, jobs: int = 8) -> str:
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    newest_header = max([os.path.getmtime(h) for h in _headers()] + [0.0])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, newest_header), srcs))
    out = ext_path()
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[gsc_amd] native extension: {out}", file=sys.stderr)
    return out


if __name__ == "__main__":
    build()
