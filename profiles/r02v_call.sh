# Final state of the round: the whole GPU suite, smoke, the default bench line
set -eo pipefail
OUT=gpurun_out/r02v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 200 python3 -u bench.py > $OUT/bench.json.log 2>&1
echo done > $OUT/DONE
