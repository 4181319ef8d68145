#!/bin/bash
# HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per run)
# over one fit of configs 3, 4 and 5.  Usage: bash tools/pmc_configs.sh <tag>
set -o pipefail
TAG=${1:-pmcc}
export TMPDIR=/tmp
for c in ${CONFIGS:-3 4 5}; do
  OUT=gpurun_out/${TAG}_c$c
  mkdir -p "$OUT"
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    echo "[pmc] $(date +%T) config $c pass $i: $grp"
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
        python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/p$i.json" 2> "$OUT/p$i.err" || exit $?
  done
done
echo "[pmc] done"
