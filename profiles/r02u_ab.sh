# One call: (1) V-cycle first sweep fused into k_axpy (DDPCA_FUSE_JAC0 1 / 0), alternating, two
# reps; (2) k_fin workgroup size 256 / 1024 with and without the two-stream split; (3) the bit-identity
# and headline parity tests
set -eo pipefail
OUT=gpurun_out/r02u
mkdir -p $OUT
export TMPDIR=/tmp
B="timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline"
for rep in 1 2; do
  for f in 0 1; do
    DDPCA_FUSE_JAC0=$f $B > $OUT/g4_fuse$f.$rep.json 2> $OUT/g4_fuse$f.$rep.err
    DDPCA_FUSE_JAC0=$f $B --groups 1 > $OUT/g1_fuse$f.$rep.json 2> $OUT/g1_fuse$f.$rep.err
  done
done
for v in "2 256" "2 1024" "1 1024" "1 256"; do
  set -- $v
  DDPCA_STREAMS=$1 DDPCA_FIN_THREADS=$2 $B > $OUT/g4_s$1_f$2.json 2> $OUT/g4_s$1_f$2.err
  DDPCA_STREAMS=$1 DDPCA_FIN_THREADS=$2 $B --groups 1 > $OUT/g1_s$1_f$2.json 2> $OUT/g1_s$1_f$2.err
done
timeout -k 10 400 python -u -m pytest tests/test_headline_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
echo done > $OUT/DONE
