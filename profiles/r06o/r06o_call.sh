#!/bin/bash
# r06o: the round's final library (block-Jacobi levels on fp32 iterate copies by default): the whole
# GPU suite, smoke(), the default bench line, one rank of the 8-, 4- and 2-rank layouts
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06o
mkdir -p $OUT
timeout -k 10 850 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=30 > $OUT/gputest.log 2>&1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 400 python3 -u profiles/one_rank_probe.py $OUT/one_rank.json --layouts 8:1,4:0,2:0 > $OUT/one_rank.log 2>&1
