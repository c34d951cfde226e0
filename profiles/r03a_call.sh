# Round 3, first call: the headline parity tests at the bench's interface density, the
# XCD-slab restriction A/B (alternating bench runs + one FETCH_SIZE pass each over
# k_restrict_lat), and the reference-vs-port CPU calibration on the GPU host itself.
set -eo pipefail
OUT=gpurun_out/r03a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_headline_gpu.py -v -s --timeout 400 --timeout-method thread > $OUT/gputest_headline.log 2>&1
B="timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline"
for x in 0 1 0 1; do
  DDPCA_XCD_RESTRICT=$x $B >> $OUT/g4_xcd$x.json 2>> $OUT/g4_xcd$x.err
done
for x in 0 1; do
  DDPCA_XCD_RESTRICT=$x timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_restrict_lat" -d $OUT/pmc_r$x -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_r$x.log 2>&1
done
timeout -k 10 400 python3 -u profiles/cpu_calibration.py 3 3 ref_harness_portable > $OUT/cpu_calibration_host.json 2> $OUT/cpu_calibration_host.err
echo done > $OUT/DONE
