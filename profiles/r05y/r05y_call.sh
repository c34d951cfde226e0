#!/bin/bash
# r05y: the one-subdomain rank's block-Jacobi set with one vs two sweeps per level (int8 copies)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05y
mkdir -p $OUT
for i in 1 2; do
  for nu in 1 2; do
    timeout -k 10 300 python3 -u profiles/one_rank_probe.py $OUT/one_rank_nu${nu}_$i.json --layouts 8:1 --options small --nu $nu --steps 20 > $OUT/one_rank_nu${nu}_$i.log 2>&1
  done
done
