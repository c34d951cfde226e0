# Round 3, call t: where the stencil-coded copies lose -- per-kernel stats with and without them
# (one stream), and the coded level copies alone (DDPCA_CODED=2: colour chunks column-indexed)
set -eo pipefail
OUT=gpurun_out/r03t
mkdir -p $OUT
export TMPDIR=/tmp
b() { timeout -k 10 240 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@"; }
DDPCA_CODED=2 b > $OUT/h_coded2only.json 2> $OUT/h_coded2only.err
b > $OUT/h_coded.json 2> $OUT/h_coded.err
DDPCA_CODED=0 b > $OUT/h_col.json 2> $OUT/h_col.err
DDPCA_CODED=2 b > $OUT/h_coded2only_b.json 2> $OUT/h_coded2only_b.err
DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_coded -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_coded.log 2>&1
DDPCA_CODED=0 DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_col -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof_col.log 2>&1
echo done > $OUT/DONE
