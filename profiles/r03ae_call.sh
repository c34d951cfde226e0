# Round 3, call ae: schedule switches re-measured on the final code, alternating in one call at 8
# subdomains per GPU: default (two streams), one stream, XCD-slab restriction, XCD-slab colour
# sweeps; and one stream vs two at 2 subdomains
set -eo pipefail
OUT=gpurun_out/r03ae
mkdir -p $OUT
export TMPDIR=/tmp
b() { timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@"; }
for rep in 1 2; do
  b > $OUT/h_default_$rep.json 2> /dev/null
  DDPCA_STREAMS=1 b > $OUT/h_onestream_$rep.json 2> /dev/null
  DDPCA_XCD_RESTRICT=1 b > $OUT/h_xcdrestrict_$rep.json 2> /dev/null
  DDPCA_GS_XCD=1 b > $OUT/h_gsxcd_$rep.json 2> /dev/null
done
for rep in 1 2; do
  b --groups 1 > $OUT/g1_default_$rep.json 2> /dev/null
  DDPCA_STREAMS=1 b --groups 1 > $OUT/g1_onestream_$rep.json 2> /dev/null
done
echo done > $OUT/DONE
