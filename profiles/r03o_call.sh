# Round 3, call o: multicolour sweep memory-layout A/B at the headline -- chunk-ordered inverses
# (default) vs by row, and XCD-slab workgroup placement -- plus one PMC FETCH pass over the
# colour sweeps of each
set -eo pipefail
OUT=gpurun_out/r03o
mkdir -p $OUT
export TMPDIR=/tmp
b() { timeout -k 10 240 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@"; }
DDPCA_GS_MINVC=0 b > $OUT/h_rowinv.json 2> $OUT/h_rowinv.err
b > $OUT/h_default.json 2> $OUT/h_default.err
DDPCA_GS_XCD=1 b > $OUT/h_xcd.json 2> $OUT/h_xcd.err
DDPCA_GS_MINVC=0 b > $OUT/h_rowinv2.json 2> $OUT/h_rowinv2.err
b > $OUT/h_default2.json 2> $OUT/h_default2.err
DDPCA_STREAMS=1 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gs" -d $OUT/pmc_default -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_default.log 2>&1
DDPCA_GS_XCD=1 DDPCA_STREAMS=1 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_gs" -d $OUT/pmc_xcd -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_xcd.log 2>&1
echo done > $OUT/DONE
