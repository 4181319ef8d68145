#!/bin/bash
# Round-3 profile set: the fp64 MFMA rate probe (random vs constant operands,
# in-kernel clock), the config-4 HBM PMC passes on the current OLS kernel, and
# rocprofv3 kernel tables of configs 3, 4, 5.  Usage: bash tools/gpu_r3_profiles.sh <tag>
set -o pipefail
TAG=${1:-r03h}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[prof] $(date +%T) mfma rate probe" &&
timeout -k 10 180 ./tools/_mfma_rate_probe > "$OUT/mfma_rate.txt" 2>&1 &&
cat "$OUT/mfma_rate.txt" &&
CONFIGS=4 bash tools/pmc_configs.sh $TAG &&
for c in 3 4 5; do
  echo "[prof] $(date +%T) rocprof c$c" &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$c" -o run -- \
      python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-parity \
      > "$OUT/bench_prof_c$c.json" 2> "$OUT/prof_c$c.err" || exit $?
done &&
echo "[prof] $(date +%T) done"
