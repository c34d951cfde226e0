#!/bin/bash
# r04a: the new transport / mass-solver / multi-rank tests, then the bench with its same-process STREAM ceiling
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_transport_gpu.py tests/test_mass_gpu.py tests/test_mcontact_gpu.py tests/test_multirank_gpu.py tests/test_headline_gpu.py tests/test_mgpis_gpu.py \
  > gpurun_out/r04a_gputest.log 2>&1 || { echo "tests failed rc=$?"; tail -50 gpurun_out/r04a_gputest.log; exit 1; }
tail -5 gpurun_out/r04a_gputest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { echo "bench failed"; tail -30 gpurun_out/r04a_bench.err; exit 1; }
cat gpurun_out/r04a_bench.json
