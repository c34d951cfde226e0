# threshold sweep of the row-split small-level SELL kernel, one box
set -eo pipefail
OUT=gpurun_out/split2
mkdir -p $OUT
for g in 4 1; do
  for t in 2048 8192 0; do
    DDPCA_SPLIT_CHUNKS=$t timeout -k 10 300 python -u bench.py --groups $g --steps 10 --no-cpu-baseline > $OUT/bench_g${g}_t${t}.log 2>&1
  done
done
echo done > $OUT/DONE
