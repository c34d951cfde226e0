# mass-CG + PCG two-stream split A/B (DDPCA_STREAMS=1 one stream, 2 default), the GPU suite, and
# the BiCGSTAB trace of the LAGRANGE CYLINDER case with and without the row-split small-level kernel
set -eo pipefail
OUT=gpurun_out/r02q
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for s in 1 2; do
    DDPCA_STREAMS=$s timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/g4_streams$s.$rep.json 2> $OUT/g4_streams$s.$rep.err
    DDPCA_STREAMS=$s timeout -k 10 240 python3 -u bench.py --groups 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/g1_streams$s.$rep.json 2> $OUT/g1_streams$s.$rep.err
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --deselect "tests/test_lagrange_gpu.py::test_lagrange_matches_reference[cylinder-hanging]" > $OUT/gputest.log 2>&1
mkdir -p $OUT/lag_a $OUT/lag_b
(cd $OUT/lag_a && DDPCA_KRYLOV_TRACE=1 DDPCA_SPLIT_CHUNKS=0 timeout -k 10 200 $GRAFT_REPO_ROOT/oracle/_ref/ref_lagrange cylinder 1 1 0 0 > out.txt 2> err.txt)
(cd $OUT/lag_b && DDPCA_KRYLOV_TRACE=1 timeout -k 10 200 $GRAFT_REPO_ROOT/oracle/_ref/ref_lagrange cylinder 1 1 0 0 > out.txt 2> err.txt)
echo done > $OUT/DONE
