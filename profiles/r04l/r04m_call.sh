#!/bin/bash
# r04m: the small-batch option set (ranks with < 4 subdomains: block Jacobi V(1,1)) against the
# multicolour set at 2 subdomains per GPU (N = 4's per-rank load) and 1 (N = 8's: --groups 1
# gives 2 subdomains; one subdomain is a worm or wheel alone, not a bench shape), alternating
name=r04m
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u profiles/sweep.py gpurun_out/${name}_small.txt "--groups 1" "--groups 1 --smoother 3 --nu 2" \
  "--groups 1" "--groups 1 --smoother 3 --nu 2" "--groups 2" "--groups 2 --smoother 1 --nu 1" "--groups 2" "--groups 2 --smoother 1 --nu 1" \
  || { echo "sweep failed"; cat gpurun_out/${name}_small.txt; exit 1; }
