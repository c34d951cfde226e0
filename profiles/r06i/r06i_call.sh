#!/bin/bash
# r06i: one rank of the 2-, 4- and 8-rank layouts (one_rank_probe.py) on the round's option sets
set -eo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06i
mkdir -p $OUT
timeout -k 10 400 python3 -u profiles/one_rank_probe.py $OUT/one_rank.json --layouts 8:1,4:0,2:0 > $OUT/one_rank.log 2>&1
timeout -k 10 300 python3 -u profiles/one_rank_probe.py $OUT/one_rank_headline.json --layouts 4:0,2:0 --options headline > $OUT/one_rank_headline.log 2>&1
