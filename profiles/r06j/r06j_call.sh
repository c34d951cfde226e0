#!/bin/bash
# r06j: the body-balance batch split into 3 or 4 parts on their own streams (DDPCA_PCG_STREAMS,
# MgpisDevice::set_split) against the two halves: bit-identity first, then the headline A/B,
# alternating in one call
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06j
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_headline_gpu.py -k "schedule_variants and (four or one-stream-small)" > $OUT/tests.log 2>&1
B="python3 -u bench.py --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling"
for i in 1 2; do
  for n in 2 3 4; do
    DDPCA_PCG_STREAMS=$n timeout -k 10 300 $B > $OUT/ab_p${n}_$i.json 2> $OUT/ab_p${n}_$i.err
    echo "{\"parts\": $n, \"line\": $(tail -1 $OUT/ab_p${n}_$i.json)}" >> $OUT/ab_all.jsonl
  done
done
