#!/bin/bash
# r06r: the round's last library (block-Jacobi fp32 copies also on levels with rotation blocks; the
# general-mesh line on precond_fp32 4): PMC traffic of the general line's roofline kernel on its new
# option set (make_traffic.py -> profiles/traffic_general.json), the whole GPU suite, smoke(), the
# default bench line
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06r
mkdir -p $OUT
G="python3 bench.py --mesh general --steps 1 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling --precond-fp32 4"
DDPCA_LATTICE=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_fetch -o run --output-format csv -- $G > $OUT/pmc_fetch.log 2>&1
DDPCA_LATTICE=0 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_write -o run --output-format csv -- $G > $OUT/pmc_write.log 2>&1
python3 profiles/make_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) --mesh general --precond-fp32 4 --out $OUT/traffic_general.json > $OUT/traffic.log 2>&1
cp $OUT/traffic_general.json profiles/traffic_general.json
timeout -k 10 850 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=30 > $OUT/gputest.log 2>&1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
find $OUT -name "*.csv" -size +20M -delete || true
