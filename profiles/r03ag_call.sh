# Round 3, call ag: the surface-mass CG's alpha inside its axpy (k_mcg_axpy_fa, one launch per CG
# iteration fewer) -- the ADMM parity suites, then A/B at 8 and 2 subdomains per GPU
set -eo pipefail
OUT=gpurun_out/r03ag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_headline_gpu.py tests/test_mcontact_gpu.py tests/test_multirank_gpu.py tests/test_hanging_gpu.py -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
b() { timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@"; }
for rep in 1 2; do
  b > $OUT/h_fa_$rep.json 2> /dev/null
  DDPCA_MCG_FUSE_ALPHA=0 b > $OUT/h_fin_$rep.json 2> /dev/null
done
for rep in 1 2; do
  b --groups 1 > $OUT/g1_fa_$rep.json 2> /dev/null
  DDPCA_MCG_FUSE_ALPHA=0 b --groups 1 > $OUT/g1_fin_$rep.json 2> /dev/null
done
echo done > $OUT/DONE
