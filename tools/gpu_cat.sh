#!/bin/bash
# Categorical-code path: its GPU parity tests, the config-3 bench in both
# layouts and a rocprofv3 kernel table.  Usage: bash tools/gpu_cat.sh <tag>
set -o pipefail
TAG=${1:-cat}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[gpu_cat] $(date +%T) pytest" &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 \
    --timeout-method thread -k "categorical or dummy" > "$OUT/pytest_cat.log" 2>&1 &&
echo "[gpu_cat] $(date +%T) bench codes" &&
timeout -k 10 300 python -u bench.py --config 3 --layout codes > "$OUT/bench_c3_codes.json" 2> "$OUT/bench_c3_codes.err" &&
echo "[gpu_cat] $(date +%T) bench dense" &&
timeout -k 10 300 python -u bench.py --config 3 --layout dense --no-cpu-baseline > "$OUT/bench_c3_dense.json" 2> "$OUT/bench_c3_dense.err" &&
echo "[gpu_cat] $(date +%T) rocprof" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o run -- \
    python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_prof_c3.json" 2> "$OUT/prof_c3.err" &&
echo "[gpu_cat] $(date +%T) done"
rc=$?
tail -15 "$OUT/pytest_cat.log"
cat "$OUT/bench_c3_codes.json" "$OUT/bench_c3_dense.json" 2>/dev/null | cut -c1-1500
exit $rc
