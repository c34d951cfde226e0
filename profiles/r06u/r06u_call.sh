#!/bin/bash
# r06u: the option sets at 8 subdomains per GPU on the last library (both on fp32 iterate copies):
# the headline's colour sweeps against two-sweep block Jacobi on every level, alternating in one call
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06u
mkdir -p $OUT
B="python3 -u bench.py --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling"
for i in 1 2; do
  timeout -k 10 300 $B > $OUT/gs_$i.json 2> $OUT/gs_$i.err
  timeout -k 10 300 $B --smoother 1 --nu 2 > $OUT/bj_$i.json 2> $OUT/bj_$i.err
done
