#!/bin/bash
# Config-5 (wide path) A/B: split Cholesky (DLSA_WIDE_SPLIT) and the MF4 Gram
# variant; wide parity tests with the split first.
# Usage: bash tools/gpu_wide_ab.sh <tag>
set -o pipefail
TAG=${1:-wideab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[wide] $(date +%T) wide parity with DLSA_WIDE_SPLIT=8"
DLSA_WIDE_SPLIT=8 timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 240 \
    --timeout-method thread -k "wide or config5 or maxiter" > "$OUT/pytest_split.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_split.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base split8 split4 gmf4; do
    L=""; E=""
    case $v in
      split8) E="DLSA_WIDE_SPLIT=8" ;;
      split4) E="DLSA_WIDE_SPLIT=4" ;;
      gmf4) L=tools/_variants/libdlsa_hip_gmf4.so ;;
    esac
    env $E DLSA_LIB=$L timeout -k 10 400 python -u bench.py --config 5 --steps 3 --no-cpu-baseline \
        > "$OUT/bench_c5_${v}_$i.json" 2> "$OUT/bench_c5_${v}_$i.err" || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('ms_per_step', v.get('avg_launch_ms', 0)), 3) for k, v in d['kernels'].items()}, d['stages_ms_per_step'])" "$OUT/bench_c5_${v}_$i.json" "c5 $v"
  done
done
