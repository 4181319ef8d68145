#!/bin/bash
# Warm-start level schedule sweep (DLSA_LEVELS / DLSA_LEVEL_TOL) on the bench
# configs: one JSON line per setting into gpurun_out/<tag>/levels.jsonl.
# Usage: bash tools/level_sweep.sh <tag>
set -o pipefail
TAG=${1:-levels}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # config levels level_tol
  local c=$1 lv=$2 lt=$3
  DLSA_LEVELS="$lv" DLSA_LEVEL_TOL="$lt" timeout -k 10 120 python -u bench.py --config "$c" \
      --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > "$OUT/tmp.json" 2>> "$OUT/levels.err" || return $?
  python - "$c" "$lv" "$lt" "$OUT/tmp.json" >> "$OUT/levels.jsonl" <<'EOF'
import json, sys
c, lv, lt, f = sys.argv[1:]
d = json.loads(open(f).read().strip().splitlines()[-1])
print(json.dumps({"config": int(c), "levels": lv, "level_tol": float(lt),
                  "ms_per_step": round(d["ms_per_step"], 2), "newton": d["newton"],
                  "dbic_support_size": d.get("dbic_support_size")}))
EOF
  tail -1 "$OUT/levels.jsonl"
}
for c in ${CONFIGS:-2 5}; do
  # space-separated schedules per config (LEVELS_C2=..., "none" = no levels)
  list_var=LEVELS_C$c
  for lv in ${!list_var:-0.0625,0.25 none 0.25 0.125,0.5 0.0625,0.25,0.5 0.03125,0.125,0.5 0.0625,0.5 0.125}; do
    [ "$lv" = none ] && lv=""
    for lt in ${TOLS:-0.1 0.03}; do
      run "$c" "$lv" "$lt" || exit $?
    done
  done
done
