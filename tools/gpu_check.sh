#!/bin/bash
# One GPU-box session: parity tests, the bench line, and a rocprofv3 kernel
# summary of a short bench run.  Usage (from the repo root, via gpurun):
#   bash tools/gpu_check.sh <tag> [pytest-args...]
# Every GPU step has its own time limit and the steps are chained with &&.
set -o pipefail
TAG=${1:-run}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
echo "[gpu_check] $(date +%T) pytest" &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "$@" \
    > "$OUT/pytest_gpu.log" 2>&1 &&
echo "[gpu_check] $(date +%T) bench" &&
timeout -k 10 420 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" &&
echo "[gpu_check] $(date +%T) rocprof" &&
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/prof.err" &&
echo "[gpu_check] $(date +%T) done"
rc=$?
tail -3 "$OUT/pytest_gpu.log"
cat "$OUT/bench.json" 2>/dev/null | head -c 3000
exit $rc
