#!/bin/bash
# r06c: fp32 stride-4 iterate copy for the fine colour sweeps (precond_fp32 = 4): V-cycle symmetry /
# solution tests, then the headline A/B against the int8 set (precond_fp32 = 3) alternating in one call
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06c
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_mgpis_gpu.py -k "fp32_iterate or symmetric_positive or int8" > $OUT/tests.log 2>&1
for i in 1 2; do
  for p in 3 4; do
    timeout -k 10 300 python3 -u bench.py --precond-fp32 $p --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_p${p}_$i.json 2> $OUT/ab_p${p}_$i.err
    tail -1 $OUT/ab_p${p}_$i.json >> $OUT/ab_all.jsonl
  done
done
