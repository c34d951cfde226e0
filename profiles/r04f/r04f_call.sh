#!/bin/bash
# r04f: colour-major fine iterate (DDPCA_GS_CM=1): bit-identity + trajectory tests, then alternating
# A/B against the natural-order sweeps at 8 subdomains per GPU
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_headline_gpu.py \
  > gpurun_out/r04f_gputest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/r04f_gputest.log; exit 1; }
tail -3 gpurun_out/r04f_gputest.log
DDPCA_GS_CM=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu \
  "tests/test_headline_gpu.py::test_headline_options_trajectory_matches_oracle" \
  > gpurun_out/r04f_gputest_cm.log 2>&1 || { echo "cm trajectory failed rc=$?"; tail -40 gpurun_out/r04f_gputest_cm.log; exit 1; }
tail -2 gpurun_out/r04f_gputest_cm.log
timeout -k 10 600 python -u profiles/sweep.py gpurun_out/r04f_ab.txt "" "DDPCA_GS_CM=1" "" "DDPCA_GS_CM=1" "" "DDPCA_GS_CM=1" \
  || { echo "sweep failed"; cat gpurun_out/r04f_ab.txt; exit 1; }
cat gpurun_out/r04f_ab.txt
