#!/bin/bash
# Ozaki exact pass, DMA lookahead A/B (DLSA_OZ_DEP) at p = 64, its GPU tests
# and the parity subset.  Usage: bash tools/gpu_oz7.sh <tag>
set -o pipefail
TAG=${1:-oz7}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[oz7] $(date +%T) ozaki tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ozaki.py -m gpu -q --timeout 120 \
    --timeout-method thread > "$OUT/pytest_ozaki.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_ozaki.log"; grep -E "^E .*(assert|Error)|FAILED" "$OUT/pytest_ozaki.log" | head -20
[ $rc -eq 0 ] || exit $rc
echo "[oz7] $(date +%T) pass A/B p=64"
timeout -k 10 300 python -u tools/pass_bench.py --n 25000000 --p 64 --K 256 --rounds 2 \
    --libs base --knobs "default;DLSA_OZ_DEP=1;DLSA_OZ=0" > "$OUT/pass_p64.jsonl" 2> "$OUT/pass_p64.err" || exit $?
cat "$OUT/pass_p64.jsonl"
echo "[oz7] $(date +%T) parity subset"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
    -k "config1 or p100 or shapes_vs_oracle or maxiter or ill_conditioned or stalled or standardized or games or misaligned or nonfinite or edge_partitions" \
    > "$OUT/pytest_subset.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_subset.log"; grep -E "^E .*(assert|Error)|FAILED" "$OUT/pytest_subset.log" | head -20
echo "[oz7] $(date +%T) done"
