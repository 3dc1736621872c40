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
import re
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("GSC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path(sanitize: bool = False) -> str:
    if sanitize:
        return os.path.join(ROOT, "build", "asan", "_native" + sysconfig.get_config_var("EXT_SUFFIX"))
    return os.path.join(ROOT, "gsc_amd", "_native" + sysconfig.get_config_var("EXT_SUFFIX"))


# Host-only AddressSanitizer + UBSan build: every -fsanitize= goes after -Xarch_host,
# so device code objects are unchanged (GPU ASan / XNACK are not available on this pool).
SAN_COMPILE = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
               "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-g"]
SAN_LINK = ["-fsanitize=address", "-fsanitize=undefined", "-shared-libsan", "-fno-gpu-sanitize"]


def _includes():
    import pybind11
    return ["-I" + CSRC, "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _flags(src: str):
    f = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result", "-Wno-unused-command-line-argument"]
    if os.sep + "sim" + os.sep in src:
        f.append("-ffp-contract=off")  # bit-exact float semantics vs the Python oracle
        # the simulator's metric atomics are issued by one lane on purpose (every lane runs the handler):
        # no wave-level reduction rewrite of uniform-address atomics
        f += ["-mllvm", "-amdgpu-atomic-optimizer-strategy=None"]
    return f


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True)
                  + glob.glob(os.path.join(CSRC, "**", "*.cpp"), recursive=True))


def _headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def _deps(path: str, seen=None) -> set:
    """Local headers a source includes, transitively (quoted includes resolved next to the includer)."""
    seen = set() if seen is None else seen
    try:
        text = open(path).read()
    except OSError:
        return seen
    for inc in _INC.findall(text):
        h = os.path.normpath(os.path.join(os.path.dirname(path), inc))
        if h not in seen and os.path.exists(h):
            seen.add(h)
            _deps(h, seen)
    return seen


def _obj(src: str, sanitize: bool = False) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "_")
    return os.path.join(BUILD + ("_asan" if sanitize else ""), rel + ".o")


def _compile(src: str, sanitize: bool = False) -> str:
    obj = _obj(src, sanitize)
    newest = max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _deps(src)])
    if os.path.exists(obj) and os.path.getmtime(obj) >= newest:
        return obj
    cmd = [HIPCC, "-c", src, "-o", obj] + _flags(src) + _includes() + (SAN_COMPILE if sanitize else [])
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose: bool = True, jobs: int = 8, sanitize: bool = False) -> str:
    os.makedirs(BUILD + ("_asan" if sanitize else ""), exist_ok=True)
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, sanitize), srcs))
    out = ext_path(sanitize)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs + (SAN_LINK if sanitize else [])
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[gsc_amd] native extension: {out}", file=sys.stderr)
    return out


if __name__ == "__main__":
    build(sanitize="--sanitize" in sys.argv)
