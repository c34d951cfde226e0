#!/bin/bash
# r05h: the whole GPU suite on the current library (timed, slowest tests listed)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05h
mkdir -p $OUT
timeout -k 10 1100 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=30 > $OUT/gputest.log 2>&1
