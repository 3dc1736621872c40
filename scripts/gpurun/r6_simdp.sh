#!/bin/bash
# Headline (Abilene, 256 envs) evidence at HEAD: simulator per-handler cycle table on the bench's 64 XCD-spread
# CUs, standalone simulator timing, plain vs forced-RCCL (world-size-1 DP) bench at 50 steps (twice each,
# interleaved), and a kernel trace of the forced-RCCL bench's timed window.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/simdp
mkdir -p $OUT
cd $R
timeout -k 10 200 python scripts/sim_throughput.py --cus 64 --cu-per-xcd 8 --steps 100 --profile > $OUT/sim_prof.txt 2>&1 || exit $?
timeout -k 10 200 python scripts/sim_throughput.py --cus 64 --cu-per-xcd 8 --steps 200 > $OUT/sim_plain.txt 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench_plain_$i.json 2> $OUT/bench_plain_$i.err || exit $?
  GSC_DIST_FORCE=1 timeout -k 10 300 python bench.py --steps 50 --warmup 5 > $OUT/bench_dp_$i.json 2> $OUT/bench_dp_$i.err || exit $?
done
export TMPDIR=/tmp
GSC_DIST_FORCE=1 GSC_PROF_WINDOW=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $OUT/prof_dp -o run -- python3 bench.py --steps 20 --warmup 5 > $OUT/prof_dp.log 2>&1
echo "rocprof rc $?" >> $OUT/prof_dp.log
exit 0
