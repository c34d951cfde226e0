#!/bin/bash
# r05a: per-launch table of the multicolour fine-level sweeps (k_gs<0|1|2>) at the bench
# configuration on the round-4 library: the library's byte model (gs_probe.py), rocprof kernel
# durations and PMC FETCH / WRITE passes (profiles/gs_table.py)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 240 python3 -u profiles/gs_probe.py --out $OUT > $OUT/probe.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/t > $OUT/trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gs" -d $OUT/pmc_fetch -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/f > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_gs" -d $OUT/pmc_write -o run --output-format csv -- python3 profiles/gs_probe.py --out $OUT/w > $OUT/pmc_write.log 2>&1
python3 profiles/gs_table.py $OUT > $OUT/gs_table.log 2>&1 || true
# keep the outputs small: the table, stats, model; drop the per-dispatch CSVs after the table
find $OUT -name "*kernel_stats.csv" -exec cp {} $OUT/ \;
find $OUT/trace $OUT/pmc_fetch $OUT/pmc_write -name "*.csv" -size +20M -delete || true
echo done > $OUT/DONE
