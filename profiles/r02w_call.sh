# (1) XCD-slab mapping of the lattice restriction (DDPCA_XCD_RESTRICT 0 / 1): alternating bench
# runs and one FETCH_SIZE pass each over k_restrict_lat; (2) single-stream kernel traces
# (DDPCA_STREAMS=1) of the final kernels at 8 and 2 subdomains per GPU
set -eo pipefail
OUT=gpurun_out/r02w
mkdir -p $OUT
export TMPDIR=/tmp
B="timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline"
for rep in 1 2; do
  for x in 0 1; do
    DDPCA_XCD_RESTRICT=$x $B > $OUT/g4_xcd$x.$rep.json 2> $OUT/g4_xcd$x.$rep.err
    DDPCA_XCD_RESTRICT=$x $B --groups 1 > $OUT/g1_xcd$x.$rep.json 2> $OUT/g1_xcd$x.$rep.err
  done
done
for x in 0 1; do
  DDPCA_XCD_RESTRICT=$x timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_restrict_lat" -d $OUT/pmc_r$x -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_r$x.log 2>&1
done
DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1
DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_g1 -o run -- python3 bench.py --groups 1 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace_g1.log 2>&1
echo done > $OUT/DONE
