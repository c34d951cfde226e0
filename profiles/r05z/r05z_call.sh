#!/bin/bash
# r05z: the tests that pin the small option set (two-sweep block Jacobi) -- its trajectory against
# the oracle, the eight-rank chain, the mass / stream variants -- on the final library
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05z
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_headline_gpu.py tests/test_transport_gpu.py -m gpu -k "not fullsize" > $OUT/tests.log 2>&1
