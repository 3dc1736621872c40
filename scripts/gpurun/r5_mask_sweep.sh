#!/bin/bash
# learner CU mask x simulator CUs at a preset (bench.py), GSC_LEARNER_MASK=0/1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/mask_${PRESET:-syn200}
mkdir -p $OUT
: > $OUT/sweep.txt
for m in ${MASKS:-1 0}; do
  for c in ${CUS:-64 96 128}; do
    GSC_LEARNER_MASK=$m timeout -k 10 300 python3 $R/bench.py --preset ${PRESET:-syn200} --steps 25 --warmup 5 --sim-cus $c > $OUT/b_${m}_$c.json 2> $OUT/b_${m}_$c.err || exit 1
    echo "learner_mask=$m sim_cus=$c $(grep -o '"value": [0-9.]*' $OUT/b_${m}_$c.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/b_${m}_$c.json)" >> $OUT/sweep.txt
  done
done
