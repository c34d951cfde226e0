# Round 3, call k: the full GPU suite on the multicolour-smoother headline option set, then the
# default bench line
set -eo pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $OUT/gputest.log 2>&1 || true
timeout -k 10 260 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done > $OUT/DONE
