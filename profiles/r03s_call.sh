set -eo pipefail
OUT=gpurun_out/r03s
mkdir -p $OUT
DDPCA_VERBOSE=1 timeout -k 10 300 python -u profiles/coded_debug.py 3 > $OUT/debug.log 2> $OUT/debug.err
echo done > $OUT/DONE
