# A/B of the V-cycle's first fine sweep fused into k_axpy (DDPCA_FUSE_JAC0=0: separate k_jac0),
# alternating runs in one call, then the bit-identity tests of the schedule variants and the
# headline / ADMM parity tests
set -eo pipefail
OUT=gpurun_out/r02s
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for f in 0 1; do
    DDPCA_FUSE_JAC0=$f timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/g4_fuse$f.$rep.json 2> $OUT/g4_fuse$f.$rep.err
    DDPCA_FUSE_JAC0=$f timeout -k 10 240 python3 -u bench.py --groups 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/g1_fuse$f.$rep.json 2> $OUT/g1_fuse$f.$rep.err
  done
done
timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py tests/test_mcontact_gpu.py tests/test_fullsize_gpu.py tests/test_mgpis_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
echo done > $OUT/DONE
