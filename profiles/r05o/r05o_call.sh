#!/bin/bash
# r05o: Chebyshev-started surface-mass solves: their tests, the schedule-variant and ADMM parity
# tests they touch, then an A/B of the headline line and of one N = 8 rank (loopback) with
# DDPCA_MASS_CHEB=0 / 1 alternating
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05o
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -v -s --timeout 450 --timeout-method thread tests/test_mass_gpu.py "tests/test_headline_gpu.py::test_schedule_variants_are_bit_identical" "tests/test_headline_gpu.py::test_headline_options_trajectory_matches_oracle" > $OUT/gputest.log 2>&1
for v in 0 1 0 1; do
  DDPCA_MASS_CHEB=$v timeout -k 10 300 python3 -u bench.py --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_cheb$v.json 2>> $OUT/ab.err
  cat $OUT/ab_cheb$v.json >> $OUT/ab_all.jsonl
done
for v in 0 1; do
  DDPCA_MASS_CHEB=$v timeout -k 10 400 python3 -u profiles/one_rank_probe.py $OUT/one_rank_cheb$v.json --layouts 8:1,4:0 > $OUT/one_rank_cheb$v.log 2>&1
done
echo done > $OUT/DONE
