#!/bin/bash
# r05k: the default bench line on the round-5 library (general-mesh object with its PMC traffic,
# cpu_baseline with the reference's own CG_SOLV)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05k
mkdir -p $OUT
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
