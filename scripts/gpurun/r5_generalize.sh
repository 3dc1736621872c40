#!/bin/bash
# held-out topology generalisation (scripts/generalize.py): PRESET, SEEDS, STEPS
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gen
mkdir -p $OUT
P=${PRESET:-syn50}
for s in ${SEEDS:-0 1 2}; do
  timeout -k 10 ${TLIMIT:-420} python3 -u $R/scripts/generalize.py --preset $P --seed $s --train-steps ${STEPS:-8000} > $OUT/${P}_s$s.txt 2>&1 || exit 1
done
