#!/bin/bash
# r06l: where the full-size iteration-4 check spends its time (its progress lines, -s); the five
# CYLINDER tests on one shared reference run
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06l
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 350 --timeout-method thread tests/test_headline_gpu.py -k fullsize_step --durations=5 > $OUT/fullsize.log 2>&1
timeout -k 10 500 python3 -u -m pytest -x -v -s --timeout 450 --timeout-method thread tests/test_mcontact_gpu.py -k "cylinder" --durations=10 > $OUT/cylinder.log 2>&1
