# A/B of the prolongation's parent-load form (DDPCA_PROLONG_SELECT build) under rocprofv3, one box
set -eo pipefail
OUT=gpurun_out/pab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/base -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/base.log 2>&1
DDPCA_AMD_LIB=$PWD/ddpca-admm_amd/libddpca_amd_psel.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/psel -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/psel.log 2>&1
echo done > $OUT/DONE
