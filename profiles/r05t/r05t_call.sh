#!/bin/bash
# r05t: the one-subdomain rank (N = 8 layout, loopback) on the multicolour vs the block-Jacobi option
# set, both on the int8 V-cycle copies, alternating
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05t
mkdir -p $OUT
for i in 1 2; do
  for o in small headline; do
    timeout -k 10 300 python3 -u profiles/one_rank_probe.py $OUT/one_rank_${o}_$i.json --layouts 8:1 --options $o --steps 20 > $OUT/one_rank_${o}_$i.log 2>&1
  done
done
