#!/bin/bash
# r05j: the band-vs-full sweeps test, then the round's PMC passes and kernel traces on the current
# library (profiles/round_profile.sh, without the bench line)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05j
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_headline_gpu.py -k "band" > $OUT/gputest.log 2>&1
timeout -k 10 1000 bash profiles/round_profile.sh r05j nobench
