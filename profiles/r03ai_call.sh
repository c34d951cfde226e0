# Round 3, call ai: the GPU test files r03ag did not cover, after the mass-CG alpha fusion
set -eo pipefail
OUT=gpurun_out/r03ai
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_double_m_gpu.py tests/test_lagrange_gpu.py tests/test_fullsize_gpu.py -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
echo done > $OUT/DONE
