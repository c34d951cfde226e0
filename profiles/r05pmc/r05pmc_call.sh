#!/bin/bash
# r05pmc: PMC traffic of the roofline kernel on the final option set (int8 V-cycle copies) for the
# headline and the general-mesh line (two passes each, make_traffic.py), then the default bench
# line reading both
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05pmc
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling > $OUT/pmc_write.log 2>&1
python3 profiles/make_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) --out $OUT/traffic.json > $OUT/traffic.log 2>&1
cp $OUT/traffic.json profiles/traffic.json
ARGS="--mesh general --no-general --no-cpu-baseline --no-stream-ceiling"
DDPCA_LATTICE=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/gpmc_fetch -o run --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 1 > $OUT/gpmc_fetch.log 2>&1
DDPCA_LATTICE=0 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/gpmc_write -o run --output-format csv -- python3 bench.py $ARGS --steps 1 --warmup 1 > $OUT/gpmc_write.log 2>&1
python3 profiles/make_traffic.py $(find $OUT/gpmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/gpmc_write -name "*counter_collection.csv" | head -1) --mesh general --out $OUT/traffic_general.json > $OUT/gtraffic.log 2>&1
cp $OUT/traffic_general.json profiles/traffic_general.json
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
find $OUT -name "*.csv" -size +20M -delete || true
