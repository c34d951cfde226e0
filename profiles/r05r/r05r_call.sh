#!/bin/bash
# r05r: block-scaled int8 V-cycle copies (precond_fp32 = 3): decode / solution tests, then the
# headline A/B against the fp16 copies, alternating in one call
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
