# A/B of the row-split small-level SELL kernel (DDPCA_SPLIT_CHUNKS=0 disables it), one box
set -eo pipefail
OUT=gpurun_out/split
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_mgpis_gpu.py tests/test_headline_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
for g in 4 1; do
  DDPCA_SPLIT_CHUNKS=0 timeout -k 10 300 python -u bench.py --groups $g --steps 10 --no-cpu-baseline > $OUT/bench_g${g}_off.log 2>&1
  timeout -k 10 300 python -u bench.py --groups $g --steps 10 --no-cpu-baseline > $OUT/bench_g${g}_on.log 2>&1
done
echo done > $OUT/DONE
