#!/bin/bash
# r04k: block-exponent fp16 on the three finest V-cycle levels by default -- the full GPU suite,
# then the default bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu --durations=30 tests \
  > gpurun_out/r04k_gputest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/r04k_gputest.log; exit 1; }
grep -a "passed\|failed" gpurun_out/r04k_gputest.log | tail -1
timeout -k 10 280 python3 -u bench.py > gpurun_out/r04k_bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/r04k_bench.log; exit 1; }
tail -1 gpurun_out/r04k_bench.log | cut -c1-300
