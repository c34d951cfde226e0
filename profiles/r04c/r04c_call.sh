#!/bin/bash
# r04c: TORSION 4 ranks with the rocSOLVER lock + the coarse-solve budget switch (TORSION, BLOCK,
# DOUBLE_M), then the round profile (PMC traffic, bench, rocprof traces at 8 and 2 subdomains)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_mcontact_gpu.py::test_torsion_known_answer tests/test_mcontact_gpu.py::test_block_patch_pressure_known_answer tests/test_double_m_gpu.py \
  > gpurun_out/r04c_gputest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/r04c_gputest.log; exit 1; }
grep -a "coarse_alt\|passed\|failed" gpurun_out/r04c_gputest.log | tail -12
bash profiles/round_profile.sh r04c || { echo "profile failed"; exit 1; }
cat gpurun_out/r04c/bench.json.log | tail -1 | cut -c1-400
