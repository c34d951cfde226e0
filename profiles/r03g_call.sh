# Round 3, call g: the multicolour smoother in the 8-subdomain headline loop (PCG capped at 200
# so a stagnating solve ends): which variant breaks down
set -eo pipefail
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
export DDPCA_PCG_MAXIT=200
for v in "3 2 2" "1 2 2" "3 1 2" "3 2 0"; do
  set -- $v
  timeout -k 10 200 python3 -u profiles/gs_debug.py 5 admm $1 $2 $3 > $OUT/admm_s$1_nu$2_musc$3.txt 2>&1
done
echo done > $OUT/DONE
