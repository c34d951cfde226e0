# Round 3, call af: one-stream kernel traces of the final code at 8 and 2 subdomains per GPU
set -eo pipefail
OUT=gpurun_out/r03af
mkdir -p $OUT
export TMPDIR=/tmp
DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.json 2> $OUT/trace.err
DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_g1 -o run --output-format csv -- python3 bench.py --groups 1 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace_g1.json 2> $OUT/trace_g1.err
echo done > $OUT/DONE
