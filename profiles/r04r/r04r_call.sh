#!/bin/bash
# r04r: the full GPU suite on the round's final library (LAGRANGE's LU coarse inverse, BLOCK
# frictionless under MGPIS restored)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu --durations=25 tests \
  > gpurun_out/r04r_gputest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/r04r_gputest.log; exit 1; }
grep -a "passed\|failed" gpurun_out/r04r_gputest.log | tail -1
