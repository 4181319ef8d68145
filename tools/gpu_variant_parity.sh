#!/bin/bash
# Parity subset of the exact (fp64) pass on a variant build.
# Usage: bash tools/gpu_variant_parity.sh <tag> <variant>
set -o pipefail
TAG=${1:-vpar}
V=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[vp] $(date +%T) parity subset on $V"
DLSA_LIB=tools/_variants/libdlsa_hip_$V.so timeout -k 10 600 python -u -m pytest tests -m gpu -v \
    --timeout 240 --timeout-method thread \
    -k "exact_pass or shapes_vs_oracle or config1 or p100 or standardized or edge_partitions or config2_shape or maxiter or ill_conditioned or ols or misaligned or games or stalled" \
    > "$OUT/pytest_$V.log" 2>&1
rc=$?; tail -4 "$OUT/pytest_$V.log"; exit $rc
