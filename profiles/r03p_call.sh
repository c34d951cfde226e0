# Round 3, call p: the hanging-level and DOUBLE_M parity tests on both option sets, the headline
# schedule variants (inverses by row / XCD slabs bit-identical)
set -eo pipefail
OUT=gpurun_out/r03p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_hanging_gpu.py tests/test_double_m_gpu.py "tests/test_headline_gpu.py::test_schedule_variants_are_bit_identical" -v -s --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1
echo done > $OUT/DONE
