#!/bin/bash
# Ozaki exact pass: stamp profile (ozprof build) + per-pass A/B against the
# fp64-MFMA pass, then the exact-pass parity subset.
# Usage: bash tools/gpu_oz2.sh <tag>
set -o pipefail
TAG=${1:-oz2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for p in 100 64; do
  echo "[oz2] $(date +%T) pass_bench p=$p"
  timeout -k 10 300 python -u tools/pass_bench.py --n 25000000 --p $p --K 256 --rounds 2 \
      --libs base,ozprof --knobs "default;DLSA_OZ=0" --hessian fp64 --max-iter 2 \
      > "$OUT/pass_p$p.jsonl" 2> "$OUT/pass_p$p.err" || exit $?
  cat "$OUT/pass_p$p.jsonl"
done
echo "[oz2] $(date +%T) parity subset"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    -k "config1 or p100 or shapes_vs_oracle or maxiter or ill_conditioned or stalled or config2_shape or edge_partitions or ols or standardized or games or exact_pass or misaligned or mixed_f32 or nonfinite or reference_signature or plain_c_abi" \
    > "$OUT/pytest_subset.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_subset.log"; grep -E "^E .*assert|FAILED" "$OUT/pytest_subset.log" | head -20
echo "[oz2] $(date +%T) done"
