# Round 3, call w: replay length with tail pacing (iters_per_graph 4 / 8 / 16), alternating, at 8
# and 2 subdomains per GPU
set -eo pipefail
OUT=gpurun_out/r03w
mkdir -p $OUT
export TMPDIR=/tmp
b() { timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@"; }
for rep in 1 2; do
  for k in 4 8 16; do
    b --iters-per-graph $k > $OUT/h_k${k}_$rep.json 2> $OUT/h_k${k}_$rep.err
  done
done
for rep in 1 2; do
  for k in 4 8 16; do
    b --groups 1 --iters-per-graph $k > $OUT/g1_k${k}_$rep.json 2> $OUT/g1_k${k}_$rep.err
  done
done
echo done > $OUT/DONE
