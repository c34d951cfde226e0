#!/bin/bash
# r05v: per-launch table of the colour sweeps on the int8 V-cycle copies (profiles/gs_table.py:
# byte model, rocprof durations, PMC FETCH / WRITE per launch)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05v
mkdir -p $OUT/gs
timeout -k 10 240 python3 -u profiles/gs_probe.py --out $OUT/gs > $OUT/gs_probe.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/gs/trace -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/gs/t > $OUT/gs_trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gs" -d $OUT/gs/pmc_fetch -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/gs/f > $OUT/gs_pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_gs" -d $OUT/gs/pmc_write -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/gs/w > $OUT/gs_pmc_write.log 2>&1
python3 profiles/gs_table.py $OUT/gs > $OUT/gs_table.log 2>&1 || true
find $OUT/gs/trace $OUT/gs/pmc_fetch $OUT/gs/pmc_write -name "*.csv" -size +20M -delete || true
