#!/bin/bash
# r05s: the whole GPU suite with the int8 V-cycle copies as the headline set, smoke(), the default
# bench line, and a kernel trace of the headline
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05s
mkdir -p $OUT
timeout -k 10 800 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=15 > $OUT/gputest.log 2>&1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling > $OUT/trace.log 2>&1
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/ \;
find $OUT/trace -name "*.csv" -size +20M -delete || true
