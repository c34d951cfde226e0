#!/bin/bash
# r06m: the whole GPU suite after the suite-time work (gather-form restriction chain, one shared
# CYLINDER reference run), smoke(), the default bench line, a rocprof kernel summary
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06m
mkdir -p $OUT
timeout -k 10 850 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=60 > $OUT/gputest.log 2>&1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling > $OUT/prof_bench.json 2> $OUT/prof_bench.err
find $OUT -name "*.csv" -size +20M -delete || true
