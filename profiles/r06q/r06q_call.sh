#!/bin/bash
# r06q: block-Jacobi fp32 copies on levels with rotation block entries (k_prolong_rot_x4): parity
# (the copy test on the general mesh, the general-mesh trajectory, the rotated hierarchies), then
# the general-mesh line on precond_fp32 4 with and without the copies, alternating in one call
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06q
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_mgpis_gpu.py -k "block_jacobi_fp32" > $OUT/tests.log 2>&1
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_rotated_transfer.py -k "general_mesh or rotated" > $OUT/tests_general.log 2>&1
G="python3 -u bench.py --mesh general --steps 10 --warmup 2 --no-cpu-baseline --no-stream-ceiling"
for i in 1 2; do
  DDPCA_BJ_X4=0 timeout -k 10 400 $G --precond-fp32 4 > $OUT/gen4_base_$i.json 2> $OUT/gen4_base_$i.err
  timeout -k 10 400 $G --precond-fp32 4 > $OUT/gen4_x4_$i.json 2> $OUT/gen4_x4_$i.err
  timeout -k 10 400 $G --precond-fp32 3 > $OUT/gen3_$i.json 2> $OUT/gen3_$i.err
done
