#!/bin/bash
# r05r: block-scaled int8 V-cycle copies (precond_fp32 = 3): decode / solution tests, the headline
# A/B against the fp16 copies alternating in one call, int8 on the fine level only, and the N = 8
# rank (block-Jacobi set) with both copies
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05r
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_mgpis_gpu.py -k "int8 or decodes or symmetric_positive" > $OUT/tests.log 2>&1
for i in 1 2; do
  for p in 2 3; do
    timeout -k 10 300 python3 -u bench.py --precond-fp32 $p --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_p${p}_$i.json 2> $OUT/ab_p${p}_$i.err
    tail -1 $OUT/ab_p${p}_$i.json >> $OUT/ab_all.jsonl
  done
done
DDPCA_Q8_LEVELS=1 timeout -k 10 300 python3 -u bench.py --precond-fp32 3 --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_p3_q1.json 2> $OUT/ab_p3_q1.err
tail -1 $OUT/ab_p3_q1.json >> $OUT/ab_all.jsonl
timeout -k 10 400 python3 -u profiles/one_rank_probe.py $OUT/one_rank_p2.json --layouts 8:1,4:0 --precond-fp32 2 > $OUT/one_rank_p2.log 2>&1
timeout -k 10 400 python3 -u profiles/one_rank_probe.py $OUT/one_rank_p3.json --layouts 8:1,4:0 --precond-fp32 3 > $OUT/one_rank_p3.log 2>&1
