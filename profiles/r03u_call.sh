# Round 3, call u: one-iteration tail graphs (pacing past the expected iteration count) --
# bit-identity against whole replays, then the A/B at 8 and 2 subdomains per GPU
set -eo pipefail
OUT=gpurun_out/r03u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "tests/test_headline_gpu.py::test_schedule_variants_are_bit_identical" -k "coded or pacing" -v -s --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
b() { timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@"; }
b > $OUT/h_tail.json 2> $OUT/h_tail.err
DDPCA_TAIL_PACING=0 b > $OUT/h_whole.json 2> $OUT/h_whole.err
b > $OUT/h_tail2.json 2> $OUT/h_tail2.err
DDPCA_TAIL_PACING=0 b > $OUT/h_whole2.json 2> $OUT/h_whole2.err
b --groups 1 > $OUT/g1_tail.json 2> $OUT/g1_tail.err
DDPCA_TAIL_PACING=0 b --groups 1 > $OUT/g1_whole.json 2> $OUT/g1_whole.err
b --groups 1 > $OUT/g1_tail2.json 2> $OUT/g1_tail2.err
DDPCA_TAIL_PACING=0 b --groups 1 > $OUT/g1_whole2.json 2> $OUT/g1_whole2.err
echo done > $OUT/DONE
