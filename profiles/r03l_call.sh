# Round 3, call l: round profile of the multicolour-smoother headline -- PMC FETCH/WRITE over the
# roofline kernel (k_sell<3>) -> profiles/traffic.json, the bench line that reads it, and the
# rocprofv3 kernel trace + stats of the default (two-stream) bench
set -eo pipefail
OUT=gpurun_out/r03l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
python3 profiles/make_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) > $OUT/traffic.log 2>&1
cp profiles/traffic.json $OUT/traffic.json
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.json 2> $OUT/trace.err
echo done > $OUT/DONE
