#!/bin/bash
# r06e: colour SSOR (smoother 4) on the fp32 iterate copy fixed (the backward sweep writes the copy
# its later colours gather); solution tests, then the headline A/B against the Gauss-Seidel pair,
# both on precond_fp32 = 4, alternating in one call
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06e
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_mgpis_gpu.py -k "colour_ssor or symmetric_positive" > $OUT/tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --precond-fp32 4 --smoother 4 --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_ssor_$i.json 2> $OUT/ab_ssor_$i.err
  tail -1 $OUT/ab_ssor_$i.json >> $OUT/ab_all.jsonl
  timeout -k 10 300 python3 -u bench.py --precond-fp32 4 --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_gs_$i.json 2> $OUT/ab_gs_$i.err
  tail -1 $OUT/ab_gs_$i.json >> $OUT/ab_all.jsonl
done
