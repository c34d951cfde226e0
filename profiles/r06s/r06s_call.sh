#!/bin/bash
# r06s: slot-loop unroll of the sweeps on the fp32 iterate copies (colour sweeps, block-Jacobi
# levels): builds with DDPCA_GS_UNROLL = 2, 3 (default) and 6, bit-identical sums; the headline and
# the N = 8 rank, alternating in one call
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06s
mkdir -p $OUT
L=ddpca-admm_amd
B="python3 -u bench.py --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling"
for i in 1 2; do
  for u in 3 2 6; do
    lib=$L/libddpca_amd.so
    if [ $u != 3 ]; then lib=$L/libu$u.so; fi
    DDPCA_AMD_LIB=$PWD/$lib timeout -k 10 300 $B > $OUT/hl_u${u}_$i.json 2> $OUT/hl_u${u}_$i.err
  done
done
for u in 3 2 6; do
  lib=$L/libddpca_amd.so
  if [ $u != 3 ]; then lib=$L/libu$u.so; fi
  DDPCA_AMD_LIB=$PWD/$lib timeout -k 10 200 python3 -u profiles/one_rank_probe.py $OUT/n8_u$u.json --layouts 8:1 > $OUT/n8_u$u.log 2>&1
done
