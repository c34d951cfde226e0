# Round 3, call j: multicolour smoother workgroup A/B (DDPCA_GS_BLOCK 256 / 64) at the headline
# and at one group, against block Jacobi V(1,1), same box
set -eo pipefail
OUT=gpurun_out/r03j
mkdir -p $OUT
export TMPDIR=/tmp
b() { timeout -k 10 240 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@"; }
b --smoother 1 --nu 1 > $OUT/h_s1.json 2> $OUT/h_s1.err
b --smoother 3 --nu 2 > $OUT/h_s3_b256.json 2> $OUT/h_s3_b256.err
DDPCA_GS_BLOCK=64 b --smoother 3 --nu 2 > $OUT/h_s3_b64.json 2> $OUT/h_s3_b64.err
b --groups 1 --smoother 1 --nu 1 > $OUT/g1_s1.json 2> $OUT/g1_s1.err
DDPCA_GS_BLOCK=64 b --groups 1 --smoother 3 --nu 2 > $OUT/g1_s3_b64.json 2> $OUT/g1_s3_b64.err
b --groups 2 --smoother 1 --nu 1 > $OUT/g2_s1.json 2> $OUT/g2_s1.err
b --groups 2 --smoother 3 --nu 2 > $OUT/g2_s3_b256.json 2> $OUT/g2_s3_b256.err
echo done > $OUT/DONE
