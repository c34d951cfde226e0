#!/bin/bash
# r05i: band-only fine sweeps on the general mesh (GsFine::band): its parity tests, then an A/B of
# the general line with DDPCA_GS_BAND=0 / 1 alternating, and the headline line (band mode must
# stay off there)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05i
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 550 --timeout-method thread tests/test_headline_gpu.py -k "general" > $OUT/gputest.log 2>&1
export DDPCA_LATTICE=0
ARGS="--mesh general --no-general --no-cpu-baseline --no-stream-ceiling"
DDPCA_VERBOSE=1 DDPCA_GS_BAND=1 timeout -k 10 300 python3 -u bench.py $ARGS --steps 3 --warmup 1 > $OUT/verbose.json 2> $OUT/verbose.err
for v in 0 1 0 1; do
  DDPCA_GS_BAND=$v timeout -k 10 300 python3 -u bench.py $ARGS > $OUT/ab_band$v.json 2>> $OUT/ab.err
  cat $OUT/ab_band$v.json >> $OUT/ab_all.jsonl
done
unset DDPCA_LATTICE
DDPCA_VERBOSE=1 timeout -k 10 300 python3 -u bench.py --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/headline.json 2> $OUT/headline.err
echo done > $OUT/DONE
