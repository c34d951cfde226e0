#!/bin/bash
# r04b: TORSION on 4 ranks with the coarse-matrix checksums, then the rest of r04a
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
mkdir -p /tmp/tors && cd /tmp/tors
DDPCA_VERBOSE=1 timeout -k 10 300 $GRAFT_REPO_ROOT/oracle/_ref/ref_torsion 2 1 2 4 > $GRAFT_REPO_ROOT/gpurun_out/r04b_torsion.log 2>&1
echo "torsion rc=$?"
cd $GRAFT_REPO_ROOT
grep -a "rank\|iters" gpurun_out/r04b_torsion.log | tail -30
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_mcontact_gpu.py tests/test_multirank_gpu.py tests/test_headline_gpu.py tests/test_mgpis_gpu.py \
  --deselect tests/test_mcontact_gpu.py::test_torsion_known_answer \
  > gpurun_out/r04b_gputest.log 2>&1 || { echo "tests failed rc=$?"; tail -50 gpurun_out/r04b_gputest.log; exit 1; }
tail -5 gpurun_out/r04b_gputest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err || { echo "bench failed"; tail -30 gpurun_out/r04b_bench.err; exit 1; }
cat gpurun_out/r04b_bench.json
