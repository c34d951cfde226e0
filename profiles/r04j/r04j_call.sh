#!/bin/bash
# r04j: block-exponent fp16 on 1 / 2 (default) / 3 V-cycle levels with the multicolour fine level
# (round 1 tuned it under block Jacobi), alternating, at 8 and 2 subdomains
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u profiles/sweep.py gpurun_out/r04j_h16.txt "" "DDPCA_H16_LEVELS=3" "DDPCA_H16_LEVELS=1" \
  "" "DDPCA_H16_LEVELS=3" "DDPCA_H16_LEVELS=1" "--groups 1" "--groups 1 DDPCA_H16_LEVELS=3" "--groups 1" "--groups 1 DDPCA_H16_LEVELS=3" \
  || { echo "sweep failed"; cat gpurun_out/r04j_h16.txt; exit 1; }
