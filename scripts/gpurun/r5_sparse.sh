#!/bin/bash
# sparse replay records: device tests, config-5 / config-4 benches (sparse default, DENSE=1 adds the dense ring),
# then the syn200 timed-window kernel table (PROF=1; last: the profiler's finalizer may crash after writing)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-sp}
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then cd $R && timeout -k 10 300 python -u -m pytest tests/test_gpu_sparse_replay.py ${EXTRA_TESTS} -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1 || exit 1; fi
for p in ${PRESETS:-syn200 syn50}; do
  timeout -k 10 400 python3 $R/bench.py --preset $p --steps ${STEPS:-25} --warmup 5 > $OUT/bench_$p.json 2> $OUT/bench_$p.err || exit 1
  if [ "${DENSE:-0}" = 1 ]; then
    GSC_SPARSE_REPLAY=0 timeout -k 10 400 python3 $R/bench.py --preset $p --steps ${STEPS:-25} --warmup 5 > $OUT/bench_${p}_dense.json 2> $OUT/bench_${p}_dense.err || exit 1
  fi
done
if [ "${PROF:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && export GSC_PROF_WINDOW=1 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d $OUT/prof -o run -- python3 $R/bench.py --preset syn200 --steps 12 --warmup 3 > $OUT/prof.log 2>&1
  python3 $R/scripts/prof_summary.py $(find $OUT/prof -name "*.db" | head -1) 12 > $OUT/prof_summary.txt 2>&1 || true
fi
exit 0
