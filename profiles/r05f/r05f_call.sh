#!/bin/bash
# r05f: the loopback timing transport (test), one rank of the N = 8 / 4 / 2 layouts alone on the GPU
# (profiles/one_rank_probe.py) with a rocprof summary of the N = 8 wheel rank, and the grid-barrier
# probe with the persistent workgroups pinned to one XCD
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05f
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 250 --timeout-method thread \
    tests/test_mcontact_gpu.py::test_loopback_timing_transport tests/test_capi.py > $OUT/gputest.log 2>&1
timeout -k 10 300 python3 -u profiles/barrier_probe.py $OUT/barrier_probe.json > $OUT/barrier_probe.log 2>&1
timeout -k 10 400 python3 -u profiles/one_rank_probe.py $OUT/one_rank.json --layouts 1:0,8:0,8:1,4:0,2:0 > $OUT/one_rank.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o n8_rank1 -- python3 -u profiles/one_rank_probe.py $OUT/one_rank_prof.json --layouts 8:1 > $OUT/prof.log 2>&1
