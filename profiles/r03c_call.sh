# Round 3, call c: the groups-1 line after the k_coarse change, then the whole GPU suite (which
# holds the tests touched this round: LAGRANGE relres / breakdown per Newton step and diag-only
# handles, CYLINDER on the library's own operator pipeline and on two ranks of one process, the
# headline coarse-correction Kx switch)
set -eo pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u bench.py --groups 1 --no-cpu-baseline > $OUT/bench_g1.json 2> $OUT/bench_g1.err
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $OUT/gputest.log 2>&1
echo done > $OUT/DONE
