#!/bin/bash
# r05q: the full-size step test with threaded oracle solves, the default bench line on the final
# library, and a kernel trace of the headline line
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05q
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 350 --timeout-method thread "tests/test_headline_gpu.py::test_headline_fullsize_step_matches_oracle" > $OUT/fullsize.log 2>&1
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling > $OUT/trace.log 2>&1
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/ \;
find $OUT/trace -name "*.csv" -size +20M -delete || true
