#!/bin/bash
# r04i: the default bench line (headline + general-mesh child + cpu_baseline + STREAM ceiling) on
# the final library, as the driver runs it
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1150 bash profiles/round_profile.sh r04i benchonly || { echo "bench failed rc=$?"; tail -30 gpurun_out/r04i/bench.json.log; exit 1; }
tail -1 gpurun_out/r04i/bench.json.log | cut -c1-600
