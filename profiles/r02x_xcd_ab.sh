# Short XCD-slab restriction A/B (DDPCA_XCD_RESTRICT 0 / 1): alternating bench runs and one
# FETCH_SIZE pass each over k_restrict_lat
set -eo pipefail
OUT=gpurun_out/r02x
mkdir -p $OUT
export TMPDIR=/tmp
B="timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline"
for x in 0 1 0 1; do
  DDPCA_XCD_RESTRICT=$x $B >> $OUT/g4_xcd$x.json 2>> $OUT/g4_xcd$x.err
done
for x in 0 1; do
  DDPCA_XCD_RESTRICT=$x timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_restrict_lat" -d $OUT/pmc_r$x -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_r$x.log 2>&1
done
echo done > $OUT/DONE
