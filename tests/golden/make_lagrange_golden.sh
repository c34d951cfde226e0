#!/bin/bash
# Records the reference's own LAGRANGE answers (Newton log, resuLagr_<ts>.txt, resuDisp) for the
# GPU test cases of tests/test_lagrange_gpu.py, by running oracle/_ref/ref_lagrange (compiled from
# /root/reference by oracle/Makefile) with DDPCA_REF_RECORD; the GPU box then replays them
# (DDPCA_REF_REPLAY) instead of re-running the reference's single-threaded Newton loop.  Runs on
# the CPU (the harness stops at the device part without a GPU, after recording).
set -u
HERE=$(cd "$(dirname "$0")" && pwd)
EXE=$HERE/../../oracle/_ref/ref_lagrange
run() {  # id args...
    local id=$1; shift
    local out=$HERE/lagrange/$id
    rm -rf "$out" && mkdir -p "$out"
    local tmp; tmp=$(mktemp -d)
    (cd "$tmp" && DDPCA_REF_RECORD="$out" OMP_NUM_THREADS=8 "$EXE" "$@" > /dev/null 2> "$tmp/err.txt")
    grep -q "recorded the reference" "$tmp/err.txt" || { echo "$id: not recorded"; tail -5 "$tmp/err.txt"; exit 1; }
    rm -rf "$tmp"
    echo "$id: $(ls "$out" | wc -l) files"
}
run mgpis-frictionless 1 1 0 0
run mgpis-coulomb-slip 1 1 0.2 2e6
run diagonal-frictionless 1 2 0 0
run cylinder-hanging cylinder 1 1 0 0
