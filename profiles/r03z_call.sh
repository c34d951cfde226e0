# Round 3, call z: the exact coarse solve's level at 8 subdomains per GPU (auto = level 1 under
# the 256 MB rule; level 2 = 8 x 80 MB dense inverses, fp32-stored 40 MB), alternating
set -eo pipefail
OUT=gpurun_out/r03z
mkdir -p $OUT
export TMPDIR=/tmp
b() { timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@"; }
for rep in 1 2; do
  b > $OUT/h_auto_$rep.json 2> $OUT/h_auto_$rep.err
  b --coarse-level 2 > $OUT/h_cl2_$rep.json 2> $OUT/h_cl2_$rep.err
done
echo done > $OUT/DONE
