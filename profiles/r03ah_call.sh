# Round 3, call ah: final-state evidence (after the mass-CG alpha fusion) -- the full GPU suite, PMC FETCH/WRITE over the roofline
# kernel (-> profiles/traffic.json), the default bench line (with the CPU baseline), the rocprofv3
# kernel trace + stats of the bench (csv, for the HIP-event cross-check) and of the one-group bench
set -eo pipefail
OUT=gpurun_out/r03ah
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $OUT/gputest.log 2>&1 || true
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
python3 profiles/make_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) > $OUT/traffic.log 2>&1
cp profiles/traffic.json $OUT/traffic.json
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_g1 -o run --output-format csv -- python3 bench.py --groups 1 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace_g1.json 2> $OUT/trace_g1.err
echo done > $OUT/DONE
