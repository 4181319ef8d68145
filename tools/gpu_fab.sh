#!/bin/bash
# Config-5 fused-pass A/B: the default library vs tools/_variants/libdlsa_hip_<v>.so
# (build with tools/build_variants.sh), kernel tables via rocprofv3.
# Usage: bash tools/gpu_fab.sh <tag> <variant>...
set -o pipefail
TAG=${1:-fab}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in default "$@"; do
  echo "[fab] $(date +%T) $v"
  if [ $v = default ]; then L=""; else L="tools/_variants/libdlsa_hip_$v.so"; fi
  DLSA_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$v" -o run -- \
      python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || exit $?
done
echo "[fab] done"
