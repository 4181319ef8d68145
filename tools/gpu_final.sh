#!/bin/bash
# Round measurement session: smoke, full GPU parity suite, the bench line of
# every config (config 2 = the driver's default line, with CPU baseline and
# parity) + rocprofv3 kernel tables, and the config-2 strong-scaling per-rank
# share at N = 8.  Usage: bash tools/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[final] $(date +%T) smoke" &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 &&
tail -1 "$OUT/smoke.log" &&
echo "[final] $(date +%T) pytest" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for c in 2 3 4 5; do
  echo "[final] $(date +%T) bench c$c" &&
  timeout -k 10 600 python -u bench.py --config $c > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" &&
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d['value'], d['roofline']['frac'], d.get('parity_rel'))" "$OUT/bench_c$c.json" "c$c" &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$c" -o run -- \
      python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/bench_prof_c$c.json" 2> "$OUT/prof_c$c.err" || exit $?
done
echo "[final] $(date +%T) strong share" &&
timeout -k 10 300 python -u bench.py --scaling strong --n 12500000 --partitions 128 --no-cpu-baseline \
    > "$OUT/bench_c2_strong_share8.json" 2> "$OUT/bench_c2_strong.err" &&
echo "[final] $(date +%T) done"
