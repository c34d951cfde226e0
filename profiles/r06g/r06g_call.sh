#!/bin/bash
# r06g: the round's library on the new headline set (precond_fp32 = 4): the whole GPU suite,
# smoke(), PMC traffic of the roofline kernel (make_traffic.py -> profiles/traffic.json), then the
# default bench line reading it
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06g
mkdir -p $OUT
timeout -k 10 850 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=15 > $OUT/gputest.log 2>&1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling > $OUT/pmc_write.log 2>&1
python3 profiles/make_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) --out $OUT/traffic.json > $OUT/traffic.log 2>&1
cp $OUT/traffic.json profiles/traffic.json
timeout -k 10 500 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
find $OUT -name "*.csv" -size +20M -delete || true
