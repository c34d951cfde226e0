#!/bin/bash
# r05u: grouped-load colour sweeps (DDPCA_GS_WIDE_MAX) -- bit-identity test, then the one-subdomain
# and two-subdomain ranks (multicolour set) and the headline with and without, alternating
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05u
mkdir -p $OUT
timeout -k 10 200 python3 -u -m pytest -x -v -s --timeout 150 --timeout-method thread tests/test_mgpis_gpu.py -k "grouped_load" > $OUT/tests.log 2>&1
for i in 1 2; do
  for w in 0 1000000000; do
    DDPCA_GS_WIDE_MAX=$w timeout -k 10 300 python3 -u profiles/one_rank_probe.py $OUT/one_rank_w${w}_$i.json --layouts 8:1,4:0 --options headline --steps 20 > $OUT/one_rank_w${w}_$i.log 2>&1
  done
done
for w in 0 1000000000; do
  DDPCA_GS_WIDE_MAX=$w timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/bench_w$w.json 2> $OUT/bench_w$w.err
  tail -1 $OUT/bench_w$w.json >> $OUT/ab_all.jsonl
done
