#!/bin/bash
# r06d: the fp32 residual for the fine restriction (precond_fp32 = 4 with / without DDPCA_GS_R32),
# the multi-rank suite with fixed-order gamma halves and LPT-packed uneven subdomains, CYLINDER /
# TORSION ranks, then the A/B: int8 (3), int8 + fp32 iterate (4, DDPCA_GS_R32=0), + fp32 residual (4)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06d
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -v -s --timeout 280 --timeout-method thread \
  tests/test_mgpis_gpu.py -k "fp32_iterate or symmetric_positive" > $OUT/tests.log 2>&1
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 280 --timeout-method thread \
  "tests/test_mcontact_gpu.py::test_cylinder_two_ranks_in_one_process" "tests/test_mcontact_gpu.py::test_torsion_known_answer" > $OUT/ranks.log 2>&1
for i in 1 2; do
  for p in 3 4r 4; do
    if [ $p = 4r ]; then
      DDPCA_GS_R32=0 timeout -k 10 300 python3 -u bench.py --precond-fp32 4 --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_p${p}_$i.json 2> $OUT/ab_p${p}_$i.err
    else
      timeout -k 10 300 python3 -u bench.py --precond-fp32 $p --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_p${p}_$i.json 2> $OUT/ab_p${p}_$i.err
    fi
    tail -1 $OUT/ab_p${p}_$i.json >> $OUT/ab_all.jsonl
  done
done
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_mgpis_gpu.py -k "colour_ssor" > $OUT/ssor_test.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --precond-fp32 4 --smoother 4 --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_ssor_$i.json 2> $OUT/ab_ssor_$i.err
  tail -1 $OUT/ab_ssor_$i.json >> $OUT/ab_all.jsonl
  timeout -k 10 300 python3 -u bench.py --precond-fp32 4 --steps 20 --warmup 3 --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_gs_$i.json 2> $OUT/ab_gs_$i.err
  tail -1 $OUT/ab_gs_$i.json >> $OUT/ab_all.jsonl
done
