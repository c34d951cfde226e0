#!/bin/bash
# r05d: TORSION's four in-process ranks (the rank harness now reports each thread's error) and
# LAGRANGE's checked coarse inverse (LU kept only at ||A^-1 A - I|| <= 1e-6)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05d
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -v -s --timeout 450 --timeout-method thread \
    tests/test_mcontact_gpu.py::test_torsion_known_answer tests/test_lagrange_gpu.py -k "torsion or block or agree" > $OUT/gputest.log 2>&1
