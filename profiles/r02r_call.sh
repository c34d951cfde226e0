# LAGRANGE with the BiCGSTAB attainable-accuracy stop (all four reference cases, row-split kernel
# on), smoke, then the round profile (PMC traffic of the roofline and V-cycle kernels, bench line,
# kernel traces at 8 and 2 subdomains per GPU)
set -eo pipefail
OUT=gpurun_out/r02r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_lagrange_gpu.py tests/test_mgpis_drivers_gpu.py -m gpu -v --timeout 400 --timeout-method thread > $OUT/gputest_lagrange.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash profiles/round_profile.sh r02r
