#!/bin/bash
# GPU session: parity suite, the default bench line (config 2, parity + CPU
# baseline), and a rocprofv3 kernel table of config 2.
# Usage: bash tools/gpu_round.sh <tag> [pytest-args...]
set -o pipefail
TAG=${1:-round}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[round] $(date +%T) pytest" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "passed|failed|error" "$OUT/pytest_gpu.log" | tail -3
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" "$OUT/pytest_gpu.log" | head -80; exit $rc; }
echo "[round] $(date +%T) bench" &&
timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo "[round] $(date +%T) rocprof" &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/bench_prof.json" 2> "$OUT/prof.err" &&
echo "[round] $(date +%T) done"
rc=$?
head -c 2500 "$OUT/bench.json"
exit $rc
