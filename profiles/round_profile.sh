#!/bin/bash
# Round-end evidence on one MI355X (run through gpurun from the repo root):
#   bench line, rocprofv3 kernel trace of the bench, two PMC passes (FETCH_SIZE, WRITE_SIZE) over
#   the roofline kernel -> profiles/traffic.json via make_traffic.py.  Every GPU step has its own
#   time limit; the script stops at the first failure.
set -eo pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
echo done > $OUT/DONE
