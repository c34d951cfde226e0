# Round 3, call aa: the row-split colour sweep (k_gs_split) for small colour launches -- the
# headline tests (reduced chain: every colour launch is small), then at 2 subdomains per GPU the
# multicolour set with and without the split against the block-Jacobi set, and at 4 the split
# forced on
set -eo pipefail
OUT=gpurun_out/r03aa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_headline_gpu.py -v -s --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
b() { timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@"; }
for rep in 1 2; do
  b --groups 1 > $OUT/g1_bj_$rep.json 2> $OUT/g1_bj_$rep.err
  b --groups 1 --smoother 3 --nu 2 > $OUT/g1_gs_split_$rep.json 2> $OUT/g1_gs_split_$rep.err
  DDPCA_GS_SPLIT_CHUNKS=0 b --groups 1 --smoother 3 --nu 2 > $OUT/g1_gs_nosplit_$rep.json 2> $OUT/g1_gs_nosplit_$rep.err
done
for rep in 1 2; do
  b --groups 2 > $OUT/g2_gs_$rep.json 2> $OUT/g2_gs_$rep.err
  DDPCA_GS_SPLIT_CHUNKS=8192 b --groups 2 > $OUT/g2_gs_split_$rep.json 2> $OUT/g2_gs_split_$rep.err
done
echo done > $OUT/DONE
