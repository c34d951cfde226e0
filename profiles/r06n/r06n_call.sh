#!/bin/bash
# r06n: fp32 iterate copies on the block-Jacobi levels (DDPCA_BJ_X4=1, precond_fp32 = 4): parity
# tests, then A/B alternating in one call -- one rank of the N = 8 layout (block Jacobi on every
# level), the headline (levels below the colour sweeps), the general-mesh line on precond_fp32 4
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06n
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_mgpis_gpu.py -k "fp32_iterate or symmetric_positive" > $OUT/tests.log 2>&1
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_headline_gpu.py -k "schedule_variants and one-stream" > $OUT/tests_default.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python3 -u profiles/one_rank_probe.py $OUT/n8_base_$i.json --layouts 8:1 > $OUT/n8_base_$i.log 2>&1
  DDPCA_BJ_X4=1 timeout -k 10 200 python3 -u profiles/one_rank_probe.py $OUT/n8_x4_$i.json --layouts 8:1 > $OUT/n8_x4_$i.log 2>&1
done
B="python3 -u bench.py --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling"
for i in 1 2; do
  timeout -k 10 300 $B > $OUT/hl_base_$i.json 2> $OUT/hl_base_$i.err
  DDPCA_BJ_X4=1 timeout -k 10 300 $B > $OUT/hl_x4_$i.json 2> $OUT/hl_x4_$i.err
done
G="python3 -u bench.py --mesh general --precond-fp32 4 --steps 10 --warmup 2 --no-cpu-baseline --no-stream-ceiling"
timeout -k 10 400 $G > $OUT/gen_base.json 2> $OUT/gen_base.err
DDPCA_BJ_X4=1 timeout -k 10 400 $G > $OUT/gen_x4.json 2> $OUT/gen_x4.err
