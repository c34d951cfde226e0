#!/bin/bash
# Round-end evidence on one MI355X (run through gpurun from the repo root):
#   two PMC passes (FETCH_SIZE, WRITE_SIZE) over the roofline kernel -> profiles/traffic.json via
#   make_traffic.py; then the bench line (which reads that traffic figure); then the rocprofv3
#   kernel trace + stats of the bench.  Every GPU step has its own time limit; the script stops at
#   the first failure.
set -eo pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
python3 profiles/make_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) > $OUT/traffic.log 2>&1
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1
echo done > $OUT/DONE
