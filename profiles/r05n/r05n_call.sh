#!/bin/bash
# r05n: the reference's CYLINDER example under the headline's V-cycle (colour GS, band mode where it applies)
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05n
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v -s --timeout 350 --timeout-method thread "tests/test_mcontact_gpu.py::test_cylinder_known_answer" > $OUT/gputest.log 2>&1
