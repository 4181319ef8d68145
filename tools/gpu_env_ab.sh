#!/bin/bash
# A/B of a runtime knob (environment variable) on the product build: the
# parity subset with the knob set, then bench.py alternated without / with it.
# Usage: bash tools/gpu_env_ab.sh <tag> <VAR=value> <config> [rounds]
set -o pipefail
TAG=${1:-envab}
KV=$2
C=${3:-2}
R=${4:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[env] $(date +%T) parity subset with $KV"
env $KV timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    -k "config1 or p100 or shapes_vs_oracle or maxiter or ill_conditioned or stalled or config2_shape or edge_partitions or distributed" \
    > "$OUT/pytest_env.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_env.log"; [ $rc -eq 0 ] || exit $rc
for i in $(seq 1 $R); do
  for arm in off on; do
    E="DLSA_AB_NONE=1"; [ $arm = on ] && E=$KV
    env $E timeout -k 10 400 python -u bench.py --config $C --steps 4 --no-cpu-baseline \
        > "$OUT/bench_c${C}_${arm}_$i.json" 2> "$OUT/bench_c${C}_${arm}_$i.err" || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v.get('ms_per_step', 0), 2) for k, v in d['kernels'].items()})" "$OUT/bench_c${C}_${arm}_$i.json" "c$C $arm"
  done
done
