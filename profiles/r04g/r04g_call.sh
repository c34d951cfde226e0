#!/bin/bash
# r04g: the full GPU suite (durations), then an A/B of one block-Jacobi sweep below the
# multicolour fine level (--nu 1) against the headline's two, and the paired mass SpMV against unpaired
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu --durations=40 tests \
  > gpurun_out/r04g_gputest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/r04g_gputest.log; exit 1; }
grep -a "passed\|failed" gpurun_out/r04g_gputest.log | tail -2
timeout -k 10 280 python -u profiles/sweep.py gpurun_out/r04g_nu.txt "" "DDPCA_MCG_PAIR=0" "--nu 1" "" "DDPCA_MCG_PAIR=0" \
  || { echo "sweep failed"; cat gpurun_out/r04g_nu.txt; exit 1; }
cat gpurun_out/r04g_nu.txt
