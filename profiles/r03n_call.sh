# Round 3, call n: smoke, the headline tests on both option sets, and the bench at 1 / 2 groups
# with the per-rank option choice (headline_options)
set -eo pipefail
OUT=gpurun_out/r03n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 500 python -u -m pytest tests/test_headline_gpu.py -v -s --timeout 400 --timeout-method thread > $OUT/gputest_headline.log 2>&1
timeout -k 10 200 python3 -u bench.py --groups 1 --no-cpu-baseline > $OUT/bench_g1.json 2> $OUT/bench_g1.err
timeout -k 10 200 python3 -u bench.py --groups 2 --no-cpu-baseline > $OUT/bench_g2.json 2> $OUT/bench_g2.err
echo done > $OUT/DONE
