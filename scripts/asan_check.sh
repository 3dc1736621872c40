#!/bin/bash
# Host AddressSanitizer + UBSan run of the native layer's CPU paths (batched simulator host path,
# launch-side code) under the CPU differential tests.  Device code is not instrumented (no GPU
# ASan on this pool); run this on CPU.
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
python "$R/gsc_amd/native/build.py" --sanitize
SO=$(ls "$R"/build/asan/_native*.so)
RT=$(find /opt/rocm/lib/llvm/lib/clang -name "libclang_rt.asan-x86_64.so" | head -1)
export GSC_NATIVE_SO="$SO"
export ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:abort_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
cd "$R"
LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" python -m pytest -q -x -p no:cacheprovider \
  tests/test_batched_sim_diff.py tests/test_large_topologies.py tests/test_oracle_golden.py "$@"
