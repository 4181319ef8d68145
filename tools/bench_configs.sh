#!/bin/bash
# Bench lines of the non-default configs (5: wide logistic, 4: OLS) and a
# rocprofv3 kernel table of each, for profiles/.  Usage: bash tools/bench_configs.sh <tag>
set -o pipefail
TAG=${1:-cfg}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in ${CONFIGS:-5 4}; do
  echo "[bench_configs] $(date +%T) config $c" &&
  timeout -k 10 300 python -u bench.py --config $c > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$c" -o run -- \
      python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_prof_c$c.json" 2> "$OUT/prof_c$c.err" || exit $?
  cat "$OUT/bench_c$c.json"
done
