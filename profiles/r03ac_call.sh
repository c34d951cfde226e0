# Round 3, call ac: the colour sweep's colour-0 launch fused into k_axpy (k_axpy_gs0) --
# bit-identity, then A/B at 8 and 4 subdomains per GPU
set -eo pipefail
OUT=gpurun_out/r03ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "tests/test_headline_gpu.py::test_schedule_variants_are_bit_identical" -v -s --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
b() { timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@"; }
for rep in 1 2; do
  b > $OUT/h_fused_$rep.json 2> $OUT/h_fused_$rep.err
  DDPCA_FUSE_GS0=0 b > $OUT/h_sep_$rep.json 2> $OUT/h_sep_$rep.err
done
for rep in 1 2; do
  b --groups 2 > $OUT/g2_fused_$rep.json 2> $OUT/g2_fused_$rep.err
  DDPCA_FUSE_GS0=0 b --groups 2 > $OUT/g2_sep_$rep.json 2> $OUT/g2_sep_$rep.err
done
echo done > $OUT/DONE
