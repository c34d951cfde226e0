#!/bin/bash
# r05w: XCD-contiguous colour-sweep chunks (DDPCA_GS_XCD=1) on the int8 copies, headline A/B
# alternating, plus the bit-identity of the solve
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05w
mkdir -p $OUT
for i in 1 2; do
  for x in 0 1; do
    DDPCA_GS_XCD=$x timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/bench_x${x}_$i.json 2> $OUT/bench_x${x}_$i.err
    tail -1 $OUT/bench_x${x}_$i.json >> $OUT/ab_all.jsonl
  done
done
