# Round 3, call i: multicolour smoother A/B -- chunk order (DDPCA_GS_TILE 0 / 1) and slot loop
# (DDPCA_GS_LOOP 1 / 2) at the headline, and one group (2 subdomains), against block Jacobi
# V(1,1), same box
set -eo pipefail
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
b() { timeout -k 10 240 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@"; }
b --smoother 1 --nu 1 > $OUT/h_s1.json 2> $OUT/h_s1.err
DDPCA_GS_TILE=0 DDPCA_GS_LOOP=1 b --smoother 3 --nu 2 > $OUT/h_s3_t0v1.json 2> $OUT/h_s3_t0v1.err
DDPCA_VERBOSE=1 DDPCA_GS_TILE=1 DDPCA_GS_LOOP=1 b --smoother 3 --nu 2 > $OUT/h_s3_t1v1.json 2> $OUT/h_s3_t1v1.err
DDPCA_GS_TILE=1 DDPCA_GS_LOOP=2 b --smoother 3 --nu 2 > $OUT/h_s3_t1v2.json 2> $OUT/h_s3_t1v2.err
b --groups 1 --smoother 1 --nu 1 > $OUT/g1_s1.json 2> $OUT/g1_s1.err
DDPCA_GS_TILE=1 DDPCA_GS_LOOP=1 b --groups 1 --smoother 3 --nu 2 > $OUT/g1_s3_t1v1.json 2> $OUT/g1_s3_t1v1.err
echo done > $OUT/DONE
