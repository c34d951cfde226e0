set -eo pipefail
OUT=gpurun_out/r02o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_g1 -o run -- python3 bench.py --groups 1 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace_g1.log 2>&1
echo done > $OUT/DONE
