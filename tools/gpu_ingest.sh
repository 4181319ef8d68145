#!/bin/bash
# Ingest + categorical checks: GPU tests, the repartition throughput, the
# config-3 bench, rocprof tables.  Usage: bash tools/gpu_ingest.sh <tag>
set -o pipefail
TAG=${1:-ing}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[gpu_ingest] $(date +%T) pytest" &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_parity.py -m gpu -x -v \
    --timeout 200 --timeout-method thread -k "ingest or repartition or csv or categorical or dummy" \
    > "$OUT/pytest.log" 2>&1 &&
echo "[gpu_ingest] $(date +%T) ingest bench" &&
timeout -k 10 300 python -u tools/ingest_bench.py > "$OUT/ingest.json" 2> "$OUT/ingest.err" &&
echo "[gpu_ingest] $(date +%T) rocprof ingest" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_ingest" -o run -- \
    python3 tools/ingest_bench.py --reps 2 > "$OUT/ingest_prof.json" 2> "$OUT/prof_ingest.err" &&
echo "[gpu_ingest] $(date +%T) bench c3" &&
timeout -k 10 300 python -u bench.py --config 3 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o run -- \
    python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_prof_c3.json" 2> "$OUT/prof_c3.err" &&
echo "[gpu_ingest] $(date +%T) done"
rc=$?
tail -25 "$OUT/pytest.log"
cat "$OUT/ingest.json" 2>/dev/null
cut -c1-600 "$OUT/bench_c3.json" 2>/dev/null
exit $rc
