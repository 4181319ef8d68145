#!/bin/bash
# Exact-pass A/B of library variants (tools/_variants/libdlsa_hip_<v>.so) in
# one process: median fp64-pass time at P = 100 (config-2 geometry, 25e6 rows).
# Usage: bash tools/gpu_pass_ab.sh <tag> <v1,v2,...> [p]
set -o pipefail
TAG=${1:-passab}
V=${2:-}
PP=${3:-100}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[ab] $(date +%T) exact pass A/B p=$PP: base,$V"
timeout -k 10 400 python -u tools/pass_bench.py --n 25000000 --p $PP --K 256 --hessian fp64 \
    --rounds 3 --libs base${V:+,$V} > "$OUT/ab_p$PP.jsonl" 2> "$OUT/ab_p$PP.err"
rc=$?; cat "$OUT/ab_p$PP.jsonl"; tail -3 "$OUT/ab_p$PP.err"; exit $rc
