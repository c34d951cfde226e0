# Round 3, call h: one-stream kernel trace of the multicolour-smoother headline (smoother 3, nu 2)
set -eo pipefail
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
DDPCA_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --smoother 3 --nu 2 > $GRAFT_REPO_ROOT/$OUT/trace.json 2> $GRAFT_REPO_ROOT/$OUT/trace.err
echo done > $GRAFT_REPO_ROOT/$OUT/DONE
