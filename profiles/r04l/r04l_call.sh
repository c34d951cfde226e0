#!/bin/bash
# r04l: sweeps below the multicolour fine level (--nu 3 vs the default 2) and the block-Jacobi
# damping (--omega-scale 1.5 / 1.9 vs 1.7), alternating, at 8 subdomains
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u profiles/sweep.py gpurun_out/r04l_nu_omega.txt "" "--nu 3" "--omega-scale 1.5" "--omega-scale 1.9" \
  "" "--nu 3" "--omega-scale 1.5" "--omega-scale 1.9" || { echo "sweep failed"; cat gpurun_out/r04l_nu_omega.txt; exit 1; }
