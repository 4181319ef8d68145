#!/bin/bash
# Ozaki exact pass: stamps + per-pass A/B, its GPU tests, the parity subset.
set -o pipefail
TAG=${1:-oz5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LIBS=${LIBS:-base,ozprof} bash tools/gpu_oz4.sh $TAG || exit $?
echo "[oz5] $(date +%T) ozaki tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ozaki.py -m gpu -v --timeout 120 \
    --timeout-method thread > "$OUT/pytest_ozaki.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_ozaki.log"; grep -E "^E .*(assert|Error)|FAILED" "$OUT/pytest_ozaki.log" | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[oz5] $(date +%T) parity subset"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
    -k "config1 or p100 or shapes_vs_oracle or maxiter or ill_conditioned or stalled or config2_shape or edge_partitions or standardized or games or misaligned or nonfinite or reference_signature or plain_c_abi" \
    > "$OUT/pytest_subset.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_subset.log"; grep -E "^E .*(assert|Error)|FAILED" "$OUT/pytest_subset.log" | head -20
echo "[oz5] $(date +%T) done"
