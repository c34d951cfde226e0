#!/bin/bash
# r04h: the grid-barrier probe (profiles/barrier_probe.py), then the round-end PMC passes (roofline kernel + fine V-cycle kernels) and the rocprofv3 kernel
# traces at 8 and 2 subdomains, on the final library (profiles/round_profile.sh, without the bench
# line, which runs as its own call)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u profiles/barrier_probe.py gpurun_out/r04h_barrier.json || { echo "barrier probe failed rc=$?"; exit 1; }
timeout -k 10 1100 bash profiles/round_profile.sh r04h nobench || { echo "round_profile failed rc=$?"; ls gpurun_out/r04h; exit 1; }
ls gpurun_out/r04h
