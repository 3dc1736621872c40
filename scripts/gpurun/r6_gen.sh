#!/bin/bash
# generalisation diagnosis (scripts/generalize.py): PRESETS, SEEDS, STEPS, EXTRA (e.g. "--on-train",
# "--schedule-threshold auto"), TAG (output suffix)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gen6
mkdir -p $OUT
for P in ${PRESETS:-type1}; do
  for s in ${SEEDS:-0 1 2}; do
    timeout -k 10 ${TLIMIT:-300} python3 -u $R/scripts/generalize.py --preset $P --seed $s --train-steps ${STEPS:-8000} $EXTRA > $OUT/${P}${TAG}_s$s.txt 2>&1 || exit 1
  done
done
