#!/bin/bash
# r05x: int8 copies with rotated hierarchies (incl. the multicolour fine level), the MGPIS suite and
# the headline trajectory tests on the rebuilt library
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05x
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rotated_transfer.py tests/test_mgpis_gpu.py "tests/test_headline_gpu.py::test_headline_options_trajectory_matches_oracle" -m gpu > $OUT/tests.log 2>&1
