"""Derived per-kernel metrics from a rocprofv3 --pmc csv (scripts/gpurun/bench_pmc.sh pass with
SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU
SQ_BUSY_CYCLES GRBM_GUI_ACTIVE).  Per dispatch (mean):
  wall      GRBM_GUI_ACTIVE / 8 XCDs (cycles), ms at the given clock
  mfma      number of v_mfma_f32_32x32x16_bf16 = SQ_VALU_MFMA_BUSY_CYCLES / 32 (the microarch guide's unit)
  TFLOP/s   mfma x 32x32x16x2 / wall time
  mfma_busy SQ_VALU_MFMA_BUSY_CYCLES / (wall x 1024 SIMDs)
  wait      SQ_WAIT_ANY / SQ_WAVE_CYCLES (share of wave time waiting)
  lds_conf  SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
``python scripts/pmc_derive.py <csv> [clock_GHz]``"""
import collections
import csv
import sys

path = sys.argv[1]
ghz = float(sys.argv[2]) if len(sys.argv) > 2 else 2.1
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.defaultdict(lambda: collections.defaultdict(set))
for row in csv.DictReader(open(path)):
    k = row["Kernel_Name"].split("(")[0].replace("void ", "")[:58]
    acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
    n[k][row["Counter_Name"]].add(row["Dispatch_Id"])
print(f"{'kernel':58s} {'wall_us':>8s} {'mfma':>9s} {'TFLOP/s':>8s} {'mfma_busy':>9s} {'wait':>5s} {'lds_conf':>8s}")
rows = []
for k, c in acc.items():
    m = {cn: v / max(1, len(n[k][cn])) for cn, v in c.items()}
    wall = m.get("GRBM_GUI_ACTIVE", 0.0) / 8
    if wall <= 0:
        continue
    t = wall / (ghz * 1e9)
    mf = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 32
    tf = mf * 32 * 32 * 16 * 2 / t / 1e12
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (wall * 1024)
    wait = m.get("SQ_WAIT_ANY", 0.0) / max(m.get("SQ_WAVE_CYCLES", 1.0), 1.0)
    lds = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(m.get("SQ_ACTIVE_INST_LDS", 1.0), 1.0)
    rows.append((t, f"{k:58s} {t * 1e6:8.1f} {mf:9.3g} {tf:8.1f} {busy:9.3f} {wait:5.2f} {lds:8.3f}"))
for _, r in sorted(rows, reverse=True):
    print(r)
