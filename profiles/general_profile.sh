#!/bin/bash
# The general-mesh line's evidence (bench.py --mesh general: contact band refined once more, hanging
# level, rotated supports, explicit transfer lists): two PMC passes (FETCH_SIZE, WRITE_SIZE) over its
# roofline kernel -> traffic_general.json (make_traffic.py --mesh general), the rocprofv3 kernel
# trace + stats of the same line, and the line itself reading that traffic figure.  Every GPU step
# has its own time limit; the script stops at the first failure.
set -eo pipefail
TAG=${1:-r05g}
OUT=gpurun_out/$TAG/general
mkdir -p $OUT
export TMPDIR=/tmp
export DDPCA_LATTICE=0
ARGS="--mesh general --no-general --no-cpu-baseline --no-stream-ceiling"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 1 > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 1 > $OUT/pmc_write.log 2>&1
python3 profiles/make_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) --mesh general --out $OUT/traffic_general.json > $OUT/traffic.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS --steps 5 --warmup 1 > $OUT/trace.log 2>&1
DDPCA_TRAFFIC_JSON=$OUT/traffic_general.json timeout -k 10 400 python3 -u bench.py $ARGS > $OUT/bench_general.json 2> $OUT/bench_general.err
find $OUT -name "*kernel_stats.csv" -exec cp {} $OUT/ \;
find $OUT/pmc_fetch $OUT/pmc_write $OUT/trace -name "*.csv" -size +20M -delete || true
echo done > $OUT/DONE
