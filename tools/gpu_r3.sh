#!/bin/bash
# Round-3 session: the GPU parity suite (new robustness / launcher tests
# first, then everything; no -x so one red test does not hide the others),
# then the config-2 bench line.  Usage: bash tools/gpu_r3.sh <tag> [bench-args...]
set -o pipefail
TAG=${1:-r03}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[r3] $(date +%T) pytest (new)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_robustness.py tests/test_gpu_distributed.py \
    -m gpu -v --timeout 240 --timeout-method thread > "$OUT/pytest_new.log" 2>&1
rc=$?; tail -15 "$OUT/pytest_new.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[r3] $(date +%T) pytest (all)"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    --deselect tests/test_gpu_robustness.py --deselect tests/test_gpu_distributed.py \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[r3] $(date +%T) bench c2"
timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" &&
head -c 600 "$OUT/bench_c2.json" && echo
