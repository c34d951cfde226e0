# Round 3, call v: warm-started surface-mass CG + its tail pacing -- the warm/cold test, the
# bit-identity variants, then the A/B at 8 and 2 subdomains per GPU
set -eo pipefail
OUT=gpurun_out/r03v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py -k "warm or pacing or one-stream or trajectory" -v -s --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
b() { timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@"; }
b > $OUT/h_warm.json 2> $OUT/h_warm.err
DDPCA_MASS_WARM=0 b > $OUT/h_cold.json 2> $OUT/h_cold.err
b > $OUT/h_warm2.json 2> $OUT/h_warm2.err
DDPCA_MASS_WARM=0 b > $OUT/h_cold2.json 2> $OUT/h_cold2.err
b --groups 1 > $OUT/g1_warm.json 2> $OUT/g1_warm.err
DDPCA_MASS_WARM=0 b --groups 1 > $OUT/g1_cold.json 2> $OUT/g1_cold.err
b --groups 1 > $OUT/g1_warm2.json 2> $OUT/g1_warm2.err
DDPCA_MASS_WARM=0 b --groups 1 > $OUT/g1_cold2.json 2> $OUT/g1_cold2.err
echo done > $OUT/DONE
