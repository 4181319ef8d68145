#!/bin/bash
# Round-3 measurement session: the GPU parity suite, the bench lines of
# configs 2 (with CPU baseline), 3, 4, 5, the N = 8 strong-scaling share of
# config 2 on one GPU, and a rocprofv3 kernel table of config 2.
# Usage: bash tools/gpu_round3.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$2" ]; then
  echo "[r3] $(date +%T) pytest"
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -4 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
echo "[r3] $(date +%T) bench c2" &&
timeout -k 10 600 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" &&
head -c 300 "$OUT/bench_c2.json" && echo &&
for c in 3 4 5; do
  echo "[r3] $(date +%T) bench c$c" &&
  timeout -k 10 600 python -u bench.py --config $c --no-cpu-baseline > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d['value'], d.get('parity_rel'), d['roofline']['frac'])" "$OUT/bench_c$c.json" c$c
done &&
echo "[r3] $(date +%T) strong share" &&
timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --no-cpu-baseline \
    > "$OUT/bench_c2_strong_share8.json" 2> "$OUT/bench_c2_strong.err" &&
echo "[r3] $(date +%T) rocprof c2" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/bench_prof_c2.json" 2> "$OUT/prof_c2.err" &&
echo "[r3] $(date +%T) done"
