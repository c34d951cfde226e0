# A/B of k_fin's workgroup size (DDPCA_FIN_THREADS 256 / 1024) with and without the two-stream
# split (DDPCA_STREAMS 2 / 1), alternating runs in one call, 8 and 2 subdomains per GPU
set -eo pipefail
OUT=gpurun_out/r02t
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "2 256" "2 1024" "1 1024" "1 256"; do
    set -- $v
    DDPCA_STREAMS=$1 DDPCA_FIN_THREADS=$2 timeout -k 10 240 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/g4_s$1_f$2.$rep.json 2> $OUT/g4_s$1_f$2.$rep.err
    DDPCA_STREAMS=$1 DDPCA_FIN_THREADS=$2 timeout -k 10 240 python3 -u bench.py --groups 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/g1_s$1_f$2.$rep.json 2> $OUT/g1_s$1_f$2.$rep.err
  done
done
echo done > $OUT/DONE
