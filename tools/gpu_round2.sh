#!/bin/bash
# Round-2 measurement session: the full GPU parity suite, the config-2 bench
# line (with CPU baseline) + rocprofv3 kernel table, the strong-scaling
# per-rank share of config 2 at N = 8 (n = 1.25e7, K = 128 on one GPU), and
# the config-5 bench + kernel table + HBM PMC passes of its pass kernels.
# Usage: bash tools/gpu_round2.sh <tag>
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p "$OUT/pmc_c5"
export TMPDIR=/tmp
echo "[r2] $(date +%T) pytest" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "[r2] $(date +%T) bench c2" &&
timeout -k 10 600 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" &&
head -c 400 "$OUT/bench_c2.json" && echo &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/bench_prof_c2.json" 2> "$OUT/prof_c2.err" &&
echo "[r2] $(date +%T) strong share" &&
timeout -k 10 300 python -u bench.py --scaling strong --n 12500000 --partitions 128 --no-cpu-baseline \
    > "$OUT/bench_c2_strong_share8.json" 2> "$OUT/bench_c2_strong.err" &&
echo "[r2] $(date +%T) bench c5" &&
timeout -k 10 420 python -u bench.py --config 5 > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run -- \
    python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/bench_prof_c5.json" 2> "$OUT/prof_c5.err" || exit $?
for grp in FETCH_SIZE WRITE_SIZE; do
  echo "[r2] $(date +%T) pmc c5 $grp"
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_c5/$grp" -o run -- \
      python3 bench.py --config 5 --steps 1 --warmup 0 --no-cpu-baseline --no-parity \
      > "$OUT/pmc_c5/$grp.json" 2> "$OUT/pmc_c5/$grp.err" || exit $?
done
echo "[r2] $(date +%T) done"
