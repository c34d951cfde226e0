#!/bin/bash
# r05p: the whole GPU suite on the library with band sweeps and Chebyshev-started mass solves
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05p
mkdir -p $OUT
timeout -k 10 1100 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=15 > $OUT/gputest.log 2>&1
