#!/bin/bash
# r04e: the full GPU suite (with durations), smoke, then the default bench (headline + general-mesh line)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu --durations=40 tests \
  > gpurun_out/r04e_gputest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/r04e_gputest.log; exit 1; }
grep -a "passed\|failed" gpurun_out/r04e_gputest.log | tail -2
