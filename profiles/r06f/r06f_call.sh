#!/bin/bash
# r06f: the reference's own ADMM iteration on the bench workload (profiles/ref_admm_time.py,
# oracle/_ref/ref_admm_time): 12 device iterations for the state, every operand dumped, the
# reference's unmodified CONTACT_ANALYSIS timed over 2 iterations on the host's 16 threads
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06f
mkdir -p $OUT
df -h /tmp > $OUT/df.txt 2>&1 || true
free -g > $OUT/free.txt 2>&1 || true
lscpu > $OUT/lscpu.txt 2>&1 || true
timeout -k 10 1100 python3 -u profiles/ref_admm_time.py $OUT/ref_admm_full.json --steps 12 --stop 2 --threads 16 > $OUT/ref_admm.log 2>&1
