# A/B of the two-stream split of the body-balance batch (DDPCA_STREAMS=1: one stream, 2: the
# default split), one box, alternating runs; the parity tests that run the split path; last, the
# LAGRANGE CYLINDER case that failed in r02o with and without the row-split small-level kernel
set -eo pipefail
OUT=gpurun_out/r02p
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for s in 1 2; do
    DDPCA_STREAMS=$s timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/g4_streams$s.$rep.json 2> $OUT/g4_streams$s.$rep.err
    DDPCA_STREAMS=$s timeout -k 10 240 python3 -u bench.py --groups 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/g1_streams$s.$rep.json 2> $OUT/g1_streams$s.$rep.err
  done
done
timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py tests/test_mcontact_gpu.py tests/test_multirank_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gputest_split.log 2>&1
DDPCA_SPLIT_CHUNKS=0 timeout -k 10 400 python -u -m pytest tests/test_lagrange_gpu.py -m gpu -x -v --timeout 380 --timeout-method thread -k cylinder > $OUT/lagrange_nosplitk.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_lagrange_gpu.py -m gpu -x -v --timeout 380 --timeout-method thread -k cylinder > $OUT/lagrange_default.log 2>&1
echo done > $OUT/DONE
