# Round 3, call c: the GPU tests touched this round -- LAGRANGE (BiCGSTAB relres / breakdown per
# Newton step, diag-only handles), the CYLINDER known answer on the library's own operator
# pipeline, the headline coarse-correction Kx switch -- then the whole GPU suite
set -eo pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_lagrange_gpu.py tests/test_mcontact_gpu.py::test_cylinder_known_answer tests/test_mcontact_gpu.py::test_cylinder_two_ranks_in_one_process "tests/test_headline_gpu.py::test_coarse_correction_kx_from_recursive_residual" -v -s --timeout 600 --timeout-method thread > $OUT/gputest_touched.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $OUT/gputest.log 2>&1
echo done > $OUT/DONE
