#!/bin/bash
# r05p: the whole GPU suite on the library with band sweeps, Chebyshev-started mass solves and the
# graphs captured at create; then smoke()
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05p
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=15 > $OUT/gputest.log 2>&1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
