#!/bin/bash
# r05y (2): block Jacobi with two / three sweeps per level against the multicolour set at 1, 2 and
# 4 subdomains per rank and on the headline (int8 copies)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05y
mkdir -p $OUT
timeout -k 10 300 python3 -u profiles/one_rank_probe.py $OUT/bj3_8.json --layouts 8:1 --options small --nu 3 --steps 20 > $OUT/bj3_8.log 2>&1
timeout -k 10 400 python3 -u profiles/one_rank_probe.py $OUT/bj2_42.json --layouts 4:0,2:0 --options small --nu 2 --steps 20 > $OUT/bj2_42.log 2>&1
timeout -k 10 400 python3 -u profiles/one_rank_probe.py $OUT/mc_42.json --layouts 4:0,2:0 --options headline --steps 20 > $OUT/mc_42.log 2>&1
timeout -k 10 300 python3 -u bench.py --smoother 1 --nu 2 --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/bench_bj2.json 2> $OUT/bench_bj2.err
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/bench_mc.json 2> $OUT/bench_mc.err
