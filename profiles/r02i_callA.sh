set -eo pipefail
OUT=gpurun_out/r02i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fullsize_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "lattice or offsets" > $OUT/test_lattice.log 2>&1
VC="k_prolong|k_restrict|k_sell<1|k_sell<2"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_sell<3" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
python3 profiles/make_traffic.py $(find $OUT/pmc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_write -name "*counter_collection.csv" | head -1) --out $OUT/traffic.json > $OUT/traffic.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$VC" -d $OUT/pmc_vc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_vc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$VC" -d $OUT/pmc_vc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/pmc_vc_write.log 2>&1
python3 profiles/pmc_kernels.py $(find $OUT/pmc_vc_fetch -name "*counter_collection.csv" | head -1) $(find $OUT/pmc_vc_write -name "*counter_collection.csv" | head -1) --out $OUT/pmc_kernels.json > $OUT/pmc_kernels.txt 2>&1
echo done > $OUT/DONE_A
