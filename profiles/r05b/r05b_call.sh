#!/bin/bash
# r05b: the general-tree coarse space on the device -- the general-mesh trajectory against the oracle
# with MULTISCALE_1 (1e-7), the headline trajectories at the tightened 1e-7; the concurrent
# factorisation test (run once); then the general-mesh bench line with the coarse space (DEHW's
# muscSett = 2, doleMcsc = 1)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05b
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_headline_gpu.py -k "general_mesh or headline_options_trajectory" tests/test_mgpis_gpu.py::test_concurrent_dense_factorisations_bit_identical -s > $OUT/gputest.log 2>&1
DDPCA_LATTICE=0 timeout -k 10 600 python3 -u bench.py --mesh general --no-general --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_general.json 2> $OUT/bench_general.err
echo done > $OUT/DONE
