#!/bin/bash
# Run GPU scripts in order; continue past test failures (rc 1) but stop on timeouts, aborts, faults.
for s in "$@"; do
  bash $s
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $s (rc=$rc)"; exit $rc; fi
done
