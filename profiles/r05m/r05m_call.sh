#!/bin/bash
# r05m: a late body-balance right-hand side of the headline run for the CPU smoother study
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05m
mkdir -p $OUT
timeout -k 10 400 python3 -u profiles/dump_rhs.py $OUT 1 0 > $OUT/dump.log 2>&1
