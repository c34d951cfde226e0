#!/bin/bash
# r05final: the whole GPU suite, smoke() and the default bench line on the round's final library
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05final
mkdir -p $OUT
timeout -k 10 800 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=10 > $OUT/gputest.log 2>&1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
