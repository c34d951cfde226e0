#!/bin/bash
# r06h: evidence on the round's headline set (precond_fp32 = 4): PMC of the V-cycle's fine-level
# transfers (pmc_kernels.py), the colour sweeps' per-launch table (gs_probe / gs_table.py), the
# whole-step cross-check -- a one-stream kernel trace and PMC passes over every kernel of one ADMM
# iteration (step_check.py); one rank per layout is r06i
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06h
mkdir -p $OUT/gs
VC="k_prolong|k_restrict|k_sell<1|k_sell<2"
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$VC" -d $OUT/pmc_vc_fetch -o run --output-format csv -- $B > $OUT/pmc_vc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$VC" -d $OUT/pmc_vc_write -o run --output-format csv -- $B > $OUT/pmc_vc_write.log 2>&1
python3 profiles/pmc_kernels.py $(find $OUT/pmc_vc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_vc_write -name "*counter_collection.csv" | head -1) --out $OUT/pmc_kernels.json > $OUT/pmc_kernels.txt 2>&1
timeout -k 10 240 python3 -u profiles/gs_probe.py --out $OUT/gs > $OUT/gs_probe.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/gs/trace -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/gs/t > $OUT/gs_trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gs" -d $OUT/gs/pmc_fetch -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/gs/f > $OUT/gs_pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_gs" -d $OUT/gs/pmc_write -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/gs/w > $OUT/gs_pmc_write.log 2>&1
python3 profiles/gs_table.py $OUT/gs > $OUT/gs_table.log 2>&1 || true
DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace1 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-general --no-stream-ceiling > $OUT/trace1.json 2> $OUT/trace1.err
DDPCA_STREAMS=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $B > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err
DDPCA_STREAMS=1 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $B > $OUT/pmc_write.json 2> $OUT/pmc_write.err
python3 profiles/step_check.py $(find $OUT/trace1 -name "*.db" | head -1) $OUT/trace1.json --fetch $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) --write $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) --pmc-bench $OUT/pmc_fetch.json --out $OUT/step_check.json > $OUT/step_check.log 2>&1 || true
find $OUT -name "*.csv" -size +20M -delete || true
find $OUT -name "*.db" -size +50M -delete || true
