#!/bin/bash
# r06a: capture-at-create + concurrent CG_SOLV, slot-summed coarse RHS (multi-rank bit-exactness),
# the four-rank TORSION with the solver lock off, then the default bench line
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06a
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 \
  tests/test_mgpis_gpu.py::test_concurrent_cg_solv_bit_identical tests/test_multirank_gpu.py \
  "tests/test_mcontact_gpu.py::test_loopback_timing_transport" \
  "tests/test_mcontact_gpu.py::test_cylinder_two_ranks_in_one_process" -s > $OUT/gputest.log 2>&1
DDPCA_SOLVER_LOCK=0 timeout -k 10 300 python3 -u -m pytest -x -v -m gpu --timeout 280 --timeout-method thread \
  "tests/test_mcontact_gpu.py::test_torsion_known_answer" -s > $OUT/torsion_lock0.log 2>&1
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
