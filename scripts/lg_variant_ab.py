#!/usr/bin/env python
"""A/B build of the native extension with gnn_lg.hip / gnn.hip taken from another commit (the rest from the working
tree): ab/lgvar/<tag>/_native*.so, loaded with GSC_NATIVE_SO=... for interleaved same-box benchmarks.

    python scripts/lg_variant_ab.py d8a4bf9
"""
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsc_amd.native import build as B  # noqa: E402


def main():
    rev = sys.argv[1]
    B.build(verbose=False)
    d = os.path.join(ROOT, "ab", "lgvar", rev)
    os.makedirs(os.path.join(d, "ops"), exist_ok=True)
    swapped = {}
    for rel in ("ops/gnn_lg.hip", "ops/gnn.hip"):
        src = os.path.join(d, rel)
        with open(src, "w") as f:
            f.write(subprocess.run(["git", "show", f"{rev}:csrc/{rel}"], capture_output=True, text=True,
                                   cwd=ROOT, check=True).stdout)
        obj = os.path.join(d, rel.replace("/", "_") + ".o")
        # headers resolve against the working tree's csrc (identical interfaces)
        cmd = [B.HIPCC, "-c", src, "-o", obj, "-I", os.path.join(B.CSRC, "ops"), "-I", B.CSRC] + \
            B._flags(src) + B._includes()
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.exit(r.stderr[-3000:])
        swapped[B._obj(os.path.join(B.CSRC, rel))] = obj
    objs = [swapped.get(B._obj(s), B._obj(s)) for s in B._sources()]
    out = os.path.join(d, "_native" + sysconfig.get_config_var("EXT_SUFFIX"))
    r = subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", out] + objs,
                       capture_output=True, text=True)
    if r.returncode != 0:
        sys.exit(r.stderr[-3000:])
    print(out)


if __name__ == "__main__":
    main()
