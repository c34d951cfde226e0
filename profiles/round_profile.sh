#!/bin/bash
# Round-end evidence on one MI355X (run through gpurun from the repo root):
#   two PMC passes (FETCH_SIZE, WRITE_SIZE) over the roofline kernel -> profiles/traffic.json via
#   make_traffic.py; two more over the V-cycle's fine-level kernels (transfers, fp16 residual and
#   sweep) -> pmc_kernels.py; then the bench line (which reads the traffic figure); then the
#   rocprofv3 kernel trace + stats of the bench, and of the one-group (2-subdomain) bench for the
#   latency-bound tail.  Every GPU step has its own time limit; the script stops at the first
#   failure.
#   Second argument: "nobench" leaves the full bench line out, "benchonly" runs only that line
#   (the two halves as separate gpurun calls when each must stay under the call limit).
set -eo pipefail
TAG=${1:-r01}
MODE=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$MODE" != benchonly ]; then
VC="k_prolong|k_restrict|k_sell<1|k_sell<2"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-general > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-general > $OUT/pmc_write.log 2>&1
python3 profiles/make_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) > $OUT/traffic.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$VC" -d $OUT/pmc_vc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-general > $OUT/pmc_vc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$VC" -d $OUT/pmc_vc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-general > $OUT/pmc_vc_write.log 2>&1
python3 profiles/pmc_kernels.py $(find $OUT/pmc_vc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_vc_write -name "*counter_collection.csv" | head -1) --out $OUT/pmc_kernels.json > $OUT/pmc_kernels.txt 2>&1
fi
if [ "$MODE" != nobench ]; then
timeout -k 10 1200 python3 -u bench.py > $OUT/bench.json.log 2>&1
fi
if [ "$MODE" != benchonly ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-general > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_g1 -o run -- python3 bench.py --groups 1 --steps 5 --warmup 1 --no-cpu-baseline --no-general > $OUT/trace_g1.log 2>&1
fi
cp profiles/traffic.json $OUT/traffic.json
echo done > $OUT/DONE
