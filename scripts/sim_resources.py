#!/usr/bin/env python
"""Register / spill / code-size table of every simulator kernel instantiation (gfx950).

Compiles ``csrc/sim/sim_kernels.hip`` device-only with the native build's flags plus
``-Rpass-analysis=kernel-resource-usage`` and prints, per kernel: VGPRs, AGPRs, SGPRs, SGPR / VGPR
spills, occupancy and code bytes (from the code object's symbol table).

    python scripts/sim_resources.py > profiles/sim_resources.txt
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gsc_amd.native import build as B  # noqa: E402


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                             text=True).stdout.split("\n")
        return {n: d for n, d in zip(names, out)}
    except OSError:
        return {n: n for n in names}


def main():
    src = os.path.join(B.CSRC, "sim", "sim_kernels.hip")
    with tempfile.TemporaryDirectory() as d:
        co = os.path.join(d, "sim.co")
        cmd = [B.HIPCC, "-c", src, "-o", co, "--cuda-device-only", "--no-gpu-bundle-output",
               "-Rpass-analysis=kernel-resource-usage"] + B._flags(src) + B._includes()
        cmd = [c for c in cmd if c != "-fPIC"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.exit(r.stderr[-4000:])
        sizes = {}
        sym = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-s", co], capture_output=True, text=True).stdout
        for line in sym.splitlines():
            f = line.split()
            if len(f) >= 8 and f[3] == "FUNC":
                sizes[f[7]] = int(f[2])
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    dem = demangle([x["name"] for x in rows])
    print(f"# {os.path.relpath(src, ROOT)}: -Rpass-analysis=kernel-resource-usage, flags {' '.join(B._flags(src))}")
    print(f"{'VGPR':>5} {'AGPR':>5} {'SGPR':>5} {'SGPRspill':>9} {'VGPRspill':>9} {'occ':>4} {'code_B':>7}  kernel")
    for x in rows:
        print(f"{x.get('VGPRs', 0):5d} {x.get('AGPRs', 0):5d} {x.get('TotalSGPRs', 0):5d} {x.get('SGPRs Spill', 0):9d} "
              f"{x.get('VGPRs Spill', 0):9d} {x.get('Occupancy [waves/SIMD]', 0):4d} {sizes.get(x['name'], 0):7d}  "
              f"{dem.get(x['name'], x['name'])}")


if __name__ == "__main__":
    main()
