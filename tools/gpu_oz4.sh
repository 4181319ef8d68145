#!/bin/bash
# Ozaki exact pass: stamp profile (ozprof build) and per-pass A/B against the
# fp64-MFMA pass in mixed mode.  Usage: bash tools/gpu_oz4.sh <tag> [p]
set -o pipefail
TAG=${1:-oz4}
P=${2:-100}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/pass_bench.py --n 25000000 --p $P --K 256 --rounds 2 \
    --libs ${LIBS:-base,ozprof} --knobs "default;DLSA_OZ=0" > "$OUT/pass_p$P.jsonl" 2> "$OUT/pass_p$P.err" || exit $?
cat "$OUT/pass_p$P.jsonl"
