#!/bin/bash
# r05e: LAGRANGE suite (checked coarse inverse reported per Newton step) and the default bench line
# with the reference's own CG_SOLV timed in cpu_baseline (reference_measured)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05e
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 550 --timeout-method thread tests/test_lagrange_gpu.py > $OUT/lagrange.log 2>&1
timeout -k 10 480 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
