# Round 3, call d: the multicolour Gauss-Seidel fine-level smoother (smoother = 3) -- the
# 8-subdomain loop (PCG capped, so a stall ends), then the headline A/B against block Jacobi
set -eo pipefail
OUT=gpurun_out/r03d
mkdir -p $OUT
export TMPDIR=/tmp
DDPCA_PCG_MAXIT=200 timeout -k 10 200 python3 -u profiles/gs_debug.py 5 admm 3 2 2 > $OUT/admm_s3_nu2_musc2.txt 2>&1
if grep -q error $OUT/admm_s3_nu2_musc2.txt; then echo "breakdown" > $OUT/STOP; exit 1; fi
for cfg in "1 1" "3 2" "3 1" "1 2"; do
  set -- $cfg
  timeout -k 10 240 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --smoother $1 --nu $2 > $OUT/bench_s$1_nu$2.json 2> $OUT/bench_s$1_nu$2.err
done
echo done > $OUT/DONE
