#!/bin/bash
# r04p: the round-end evidence set on the final library (block-exponent fp16 on three levels, the
# small-batch threshold at one subdomain per rank): PMC passes, the default bench line, rocprof
# kernel traces at 8 and 2 subdomains (profiles/round_profile.sh)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1150 bash profiles/round_profile.sh r04p || { echo "round_profile failed rc=$?"; ls gpurun_out/r04p; exit 1; }
tail -1 gpurun_out/r04p/bench.json.log | cut -c1-300
