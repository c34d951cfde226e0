#!/bin/bash
# r04d: fused PCG scalar updates (bit-identity against the k_fin launches, trajectory parity), the
# colour sweeps' occupancy cap and the general-mesh trajectory test; alternating A/B runs: new
# default / DDPCA_FUSED_FIN=0 / the library before both changes (libddpca_ab.so), at 8 and 2
# subdomains per GPU; then the full-size general-mesh bench line on its own
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_headline_gpu.py tests/test_mgpis_gpu.py \
  > gpurun_out/r04d_gputest.log 2>&1 || { echo "tests failed rc=$?"; tail -60 gpurun_out/r04d_gputest.log; exit 1; }
tail -3 gpurun_out/r04d_gputest.log
OLD=DDPCA_AMD_LIB=ddpca-admm_amd/libddpca_ab.so
timeout -k 10 700 python -u profiles/sweep.py gpurun_out/r04d_ab.txt "" "DDPCA_FUSED_FIN=0" "$OLD" \
  "--groups 1" "DDPCA_FUSED_FIN=0 --groups 1" "$OLD --groups 1" \
  || { echo "sweep failed"; cat gpurun_out/r04d_ab.txt; exit 1; }
cat gpurun_out/r04d_ab.txt
DDPCA_LATTICE=0 timeout -k 10 600 python -u bench.py --mesh general --no-general --no-cpu-baseline --steps 5 --warmup 1 \
  > gpurun_out/r04d_general.json 2> gpurun_out/r04d_general.err || { echo "general failed"; tail -30 gpurun_out/r04d_general.err; exit 1; }
cut -c1-1500 gpurun_out/r04d_general.json
