#!/bin/bash
# r05c: LATIN's DOUBLE_M on non-nested coarse contact nodes (BLOCK's budget-forced DOUBLE_M, CYLINDER
# on two ranks incl. owners 0011), the DOUBLE_M suites, and the concurrent factorisation test (once)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05c
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 350 --timeout-method thread tests/test_mgpis_gpu.py::test_concurrent_dense_factorisations_bit_identical > $OUT/concurrent.log 2>&1
timeout -k 10 1000 python3 -u -m pytest -v -s --timeout 400 --timeout-method thread tests/test_double_m_gpu.py tests/test_mcontact_gpu.py > $OUT/gputest.log 2>&1
echo done > $OUT/DONE
