#!/usr/bin/env python
"""A/B builds of the native extension whose simulator step kernel has a capped SGPR budget (GSC_SIM_MAX_SGPR): more
SGPR spills (to VGPR lanes) in the same code, to measure what a spill costs.  Writes ab/simvar/sgpr<N>/_native*.so
(load one with GSC_NATIVE_SO=...) and prints the headline kernel's resource line per variant.

    python scripts/sim_sgpr_ab.py 96 80
"""
import os
import re
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsc_amd.native import build as B  # noqa: E402


def main():
    B.build(verbose=False)  # the default objects
    src = os.path.join(B.CSRC, "sim", "sim_kernels.hip")
    objs = [B._obj(s) for s in B._sources()]
    for n in [int(x) for x in sys.argv[1:]]:
        d = os.path.join(ROOT, "ab", "simvar", f"sgpr{n}")
        os.makedirs(d, exist_ok=True)
        obj = os.path.join(d, "sim_kernels.o")
        cmd = [B.HIPCC, "-c", src, "-o", obj, f"-DGSC_SIM_MAX_SGPR={n}", "-Rpass-analysis=kernel-resource-usage"] + \
            B._flags(src) + B._includes()
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.exit(r.stderr[-3000:])
        # resource line of the headline kernel <2, 1, false, true>
        blocks = r.stderr.split("Function Name: ")
        for b in blocks:
            if b.startswith("_ZN3gsc15sim_step_kernelILi2ELi1ELb0ELb1EEEvNS_7SimArgsE"):
                vals = dict(re.findall(r"remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)", b))
                print(f"sgpr cap {n}: SGPRs {vals.get('TotalSGPRs')} spill {vals.get('SGPRs Spill')} VGPRs "
                      f"{vals.get('VGPRs')} VGPR spill {vals.get('VGPRs Spill')} occupancy {vals.get('Occupancy [waves/SIMD]')}")
        mine = [obj if o == B._obj(src) else o for o in objs]
        out = os.path.join(d, "_native" + sysconfig.get_config_var("EXT_SUFFIX"))
        r = subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", "-o", out] + mine,
                           capture_output=True, text=True)
        if r.returncode != 0:
            sys.exit(r.stderr[-3000:])
        print(out)


if __name__ == "__main__":
    main()
