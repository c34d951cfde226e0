#!/bin/bash
# r06v: rocprofv3 kernel summary of the default bench command on the round's last library (the
# roofline kernel's rocprof average against the line's own HIP-event figure in the same run)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06v
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-general > $OUT/bench.json 2> $OUT/bench.err
python3 profiles/roofline_check_csv.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) $OUT/bench.json > $OUT/roofline_check.txt 2>&1 || true
find $OUT -name "*kernel_trace.csv" -size +20M -delete || true
