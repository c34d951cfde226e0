# Round 3, call m: whole-step cross-check of the multicolour-smoother headline (one-stream kernel
# trace + PMC FETCH_SIZE / WRITE_SIZE over every kernel of one ADMM iteration, profiles/step_check.py)
# and the one-group (2-subdomain) one-stream trace for the tail
set -eo pipefail
OUT=gpurun_out/r03m
mkdir -p $OUT
export TMPDIR=/tmp
DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace1.json 2> $OUT/trace1.err
DDPCA_STREAMS=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err
DDPCA_STREAMS=1 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.json 2> $OUT/pmc_write.err
python3 profiles/step_check.py $(find $OUT/trace1 -name "*.db" | head -1) $OUT/trace1.json --fetch $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) --write $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) --pmc-bench $OUT/pmc_fetch.json --out $OUT/step_check.json > $OUT/step_check.log 2>&1 || true
DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_g1 -o run -- python3 bench.py --groups 1 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace_g1.json 2> $OUT/trace_g1.err
echo done > $OUT/DONE
