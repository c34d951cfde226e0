# Round 3, call y: the MGPIS suite after the table mode's products took the streamed kernels'
# explicit contraction (y = Kx bit-identical again)
set -eo pipefail
OUT=gpurun_out/r03y
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_mgpis_gpu.py -v --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1
echo done > $OUT/DONE
