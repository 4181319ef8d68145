#!/bin/bash
# Quick GPU session: parity tests, then bench + rocprof kernel table of the
# configs in $CONFIGS (default "2 4").  Usage: bash tools/gpu_quick.sh <tag> [pytest-args...]
set -o pipefail
TAG=${1:-quick}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[gpu_quick] $(date +%T) pytest" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "$@" \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
for c in ${CONFIGS:-2 4}; do
  echo "[gpu_quick] $(date +%T) config $c" &&
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$c" -o run -- \
      python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_prof_c$c.json" 2> "$OUT/prof_c$c.err" || exit $?
  head -c 1500 "$OUT/bench_c$c.json"; echo
done
