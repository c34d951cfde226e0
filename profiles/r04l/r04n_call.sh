#!/bin/bash
# r04n: one subdomain per GPU -- the multicolour vs the block-Jacobi option set on one full-size
# subdomain solve (profiles/one_sub_probe.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u profiles/one_sub_probe.py gpurun_out/r04n_one_sub.json ${VARIANTS:-} || { echo "probe failed rc=$?"; exit 1; }
