#!/bin/bash
# r06t: the tree as committed at the end of round 6 -- the whole GPU suite, smoke() and the default
# bench line, as the driver runs them
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06t
mkdir -p $OUT
timeout -k 10 850 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=30 > $OUT/gputest.log 2>&1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
