#!/bin/bash
# r05ab: kernel stats of the N = 8 rank on the final small set (two-sweep block Jacobi, int8), and
# the general-mesh line on that set against its own (multicolour band) for the record
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05ab
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/n8 -o run --output-format csv -- python3 profiles/one_rank_probe.py $OUT/n8_rank1.json --layouts 8:1 --steps 10 > $OUT/n8.log 2>&1
find $OUT/n8 -name "*kernel_stats.csv" -exec cp {} $OUT/n8_rank1_kernel_stats.csv \;
find $OUT/n8 -name "*.csv" -size +20M -delete || true
DDPCA_LATTICE=0 timeout -k 10 400 python3 -u bench.py --mesh general --no-general --no-cpu-baseline --no-stream-ceiling --smoother 1 --nu 2 --steps 10 > $OUT/general_bj2.json 2> $OUT/general_bj2.err
DDPCA_LATTICE=0 timeout -k 10 400 python3 -u bench.py --mesh general --no-general --no-cpu-baseline --no-stream-ceiling --steps 10 > $OUT/general_mc.json 2> $OUT/general_mc.err
