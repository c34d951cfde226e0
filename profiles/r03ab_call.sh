# Round 3, call ab: MONITOR pair norms batched into two launches -- bit-identity, then A/B at 8
# subdomains per GPU
set -eo pipefail
OUT=gpurun_out/r03ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "tests/test_headline_gpu.py::test_schedule_variants_are_bit_identical" -v -s --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
b() { timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@"; }
for rep in 1 2; do
  b > $OUT/h_batched_$rep.json 2> $OUT/h_batched_$rep.err
  DDPCA_NORMS_BATCHED=0 b > $OUT/h_pairs_$rep.json 2> $OUT/h_pairs_$rep.err
done
echo done > $OUT/DONE
