#!/bin/bash
# r05l: the device's PCG iteration counts in the last timed ADMM iteration (the state cpu_baseline
# prices with the reference's own CG_SOLV: 15 iterations there)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05l
mkdir -p $OUT
timeout -k 10 400 python3 -u bench.py --no-general --no-stream-ceiling > $OUT/bench.json 2> $OUT/bench.err
