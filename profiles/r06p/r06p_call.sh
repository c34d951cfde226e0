#!/bin/bash
# r06p: the whole-step cross-check on the round's last library (block-Jacobi fp32 copies in): a
# one-stream kernel trace and PMC passes over every kernel of one ADMM iteration (step_check.py);
# the N = 8 rank's kernel summary (one_rank_probe under rocprofv3)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06p
mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling"
DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling > $OUT/trace1.json 2> $OUT/trace1.err
DDPCA_STREAMS=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $B > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err
DDPCA_STREAMS=1 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $B > $OUT/pmc_write.json 2> $OUT/pmc_write.err
python3 profiles/step_check.py $(find $OUT/trace1 -name "*.db" | head -1) $OUT/trace1.json --fetch $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) --write $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) --pmc-bench $OUT/pmc_fetch.json --out $OUT/step_check.json > $OUT/step_check.log 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/n8 -o run --output-format csv -- python3 -u profiles/one_rank_probe.py $OUT/n8_rank1.json --layouts 8:1 > $OUT/n8.log 2>&1
find $OUT -name "*.csv" -size +20M -delete || true
find $OUT -name "*.db" -size +50M -delete || true
