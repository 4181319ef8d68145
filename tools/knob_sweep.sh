#!/bin/bash
# bench.py under several pass knobs (env), one line each.  Usage:
#   bash tools/knob_sweep.sh <tag> "<bench args>" "ENV=V ENV2=V" "ENV=V" ...
set -o pipefail
TAG=$1; ARGS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for k in "$@"; do
  i=$((i+1))
  echo "[sweep] $(date +%T) $k"
  env $k timeout -k 10 200 python -u bench.py $ARGS --no-cpu-baseline > "$OUT/k$i.json" 2> "$OUT/k$i.err" || exit $?
  python3 -c "import json,sys; d=json.load(open('$OUT/k$i.json')); print('$k', round(d['ms_per_step'],2), {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)),3) for k,v in d['kernels'].items()})"
done
