# Round 3, call r: stencil-coded V-cycle copies -- bit-identity against the column-indexed copies
# on both option sets, the headline parity tests, smoke; then the headline A/B (alternating runs)
# at 8 and 2 subdomains per GPU
set -eo pipefail
OUT=gpurun_out/r03r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "tests/test_headline_gpu.py::test_schedule_variants_are_bit_identical" -k column -v -s --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
b() { timeout -k 10 240 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@"; }
b > $OUT/h_coded.json 2> $OUT/h_coded.err
DDPCA_CODED=0 b > $OUT/h_col.json 2> $OUT/h_col.err
b > $OUT/h_coded2.json 2> $OUT/h_coded2.err
DDPCA_CODED=0 b > $OUT/h_col2.json 2> $OUT/h_col2.err
b --groups 1 > $OUT/g1_coded.json 2> $OUT/g1_coded.err
DDPCA_CODED=0 b --groups 1 > $OUT/g1_col.json 2> $OUT/g1_col.err
b --groups 1 > $OUT/g1_coded2.json 2> $OUT/g1_coded2.err
echo done > $OUT/DONE
