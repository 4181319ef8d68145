#!/bin/bash
# A/B of exact-pass (fp64) kernel variants selected by env knobs, plus the
# GPU parity suite.  Usage: bash tools/gpu_ab.sh <tag> "<knobs1>;<knobs2>;..."
set -o pipefail
TAG=${1:-ab}
KNOBS=${2:-default}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[ab] $(date +%T) pytest" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "[ab] $(date +%T) pass_bench fp64" &&
timeout -k 10 300 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --hessian fp64 --rounds 3 \
    --knobs "$KNOBS" > "$OUT/pass_fp64.jsonl" 2> "$OUT/pass_fp64.err" && cat "$OUT/pass_fp64.jsonl" &&
IFS=';' read -ra KS <<< "$KNOBS" &&
for k in "${KS[@]}"; do
  env $( [ "$k" = default ] || echo "${k//,/ }" ) timeout -k 10 300 python -u bench.py --config 4 --no-cpu-baseline \
      > "$OUT/c4_${k//[=,]/_}.json" 2> "$OUT/c4.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], {k:v.get('avg_launch_ms') for k,v in d['kernels'].items()})" "$OUT/c4_${k//[=,]/_}.json" "$k"
done
