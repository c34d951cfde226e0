# Round 3, call f: the multicolour smoother at gl = 4 and 5 (MGPIS per subdomain, capped at 300)
set -eo pipefail
OUT=gpurun_out/r03f
mkdir -p $OUT
export TMPDIR=/tmp
DDPCA_VERBOSE=1 timeout -k 10 300 python3 -u profiles/gs_debug.py 4 mgpis > $OUT/mgpis_gl4.txt 2>&1
DDPCA_VERBOSE=1 timeout -k 10 500 python3 -u profiles/gs_debug.py 5 mgpis > $OUT/mgpis_gl5.txt 2>&1
echo done > $OUT/DONE
