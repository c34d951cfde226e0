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
timeout -k 10 400 python3 -u profiles/one_rank_probe.py $OUT/one_rank.json --layouts 1:0,8:1,8:0,4:0,2:0 > $OUT/one_rank.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o n8_rank1 -- python3 -u profiles/one_rank_probe.py $OUT/one_rank_prof.json --layouts 8:1 > $OUT/prof.log 2>&1
# A/B of the XCD-contiguous chunk ranges of the colour sweeps (DDPCA_GS_XCD), alternating
for v in 0 1 0 1; do
  DDPCA_GS_XCD=$v timeout -k 10 300 python3 -u bench.py --no-general --no-cpu-baseline --no-stream-ceiling > $OUT/ab_xcd$v.json 2>> $OUT/ab.err
  cat $OUT/ab_xcd$v.json >> $OUT/ab_all.jsonl
done
# the per-launch table of the sweeps with the XCD mapping (r05a's recipe)
timeout -k 10 240 python3 -u profiles/gs_probe.py --out $OUT/gs > $OUT/gs_probe.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/gs/trace -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/gs/t > $OUT/gs_trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gs" -d $OUT/gs/pmc_fetch -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/gs/f > $OUT/gs_pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_gs" -d $OUT/gs/pmc_write -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/gs/w > $OUT/gs_pmc_write.log 2>&1
python3 profiles/gs_table.py $OUT/gs > $OUT/gs_table.log 2>&1 || true
find $OUT/gs -name "*kernel_stats.csv" -exec cp {} $OUT/gs/ \; || true
find $OUT/gs/trace $OUT/gs/pmc_fetch $OUT/gs/pmc_write $OUT/prof -name "*.csv" -size +20M -delete || true
echo done > $OUT/DONE
