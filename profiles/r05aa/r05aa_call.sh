#!/bin/bash
# r05aa: how many of the finest levels take the int8 copy (DDPCA_H16_LEVELS 2 / 3 / 4) and PCG
# iterations per graph replay (4 / 6) on the headline, alternating with the default
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05aa
mkdir -p $OUT
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling ${BARGS:-} > $OUT/$name.json 2> $OUT/$name.err
  echo "$name $(tail -1 $OUT/$name.json)" >> $OUT/ab_all.txt
}
run base1 DDPCA_H16_LEVELS=3
run h2 DDPCA_H16_LEVELS=2
run h4 DDPCA_H16_LEVELS=4
run base2 DDPCA_H16_LEVELS=3
BARGS="--iters-per-graph 6" run g6 DDPCA_H16_LEVELS=3
run base3 DDPCA_H16_LEVELS=3
