#!/bin/bash
# Measurement session: variant A/B of the passes, HBM-traffic PMC passes of
# every config's roofline kernel (FETCH_SIZE, WRITE_SIZE: one counter group
# per run), and the bench line + rocprofv3 kernel table of configs 3, 4, 5.
# Usage: bash tools/gpu_measure.sh <tag> [libs]
set -o pipefail
TAG=${1:-meas}
LIBS=${2:-base}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$LIBS" != none ]; then
echo "[meas] $(date +%T) pass A/B ($LIBS)" &&
timeout -k 10 300 python -u tools/pass_bench.py --n 50000000 --p 100 --K 512 --rounds 3 \
    --libs "$LIBS" > "$OUT/pass_mixed.jsonl" 2> "$OUT/pass_mixed.err" && cat "$OUT/pass_mixed.jsonl" &&
timeout -k 10 300 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --rounds 3 --hessian fp64 \
    --libs "$LIBS" > "$OUT/pass_fp64.jsonl" 2> "$OUT/pass_fp64.err" && cat "$OUT/pass_fp64.jsonl" || exit $?
fi
for c in 2 3 4 5; do
  mkdir -p "$OUT/pmc_c$c"
  for grp in FETCH_SIZE WRITE_SIZE; do
    echo "[meas] $(date +%T) pmc config $c $grp"
    timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc_c$c/$grp" -o run -- \
        python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-parity \
        > "$OUT/pmc_c$c/$grp.json" 2> "$OUT/pmc_c$c/$grp.err" || exit $?
  done
done
for c in 3 4 5; do
  echo "[meas] $(date +%T) bench config $c" &&
  timeout -k 10 420 python -u bench.py --config $c > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err" &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c$c" -o run -- \
      python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline --no-parity \
      > "$OUT/bench_prof_c$c.json" 2> "$OUT/prof_c$c.err" || exit $?
  head -c 600 "$OUT/bench_c$c.json"; echo
done
echo "[meas] $(date +%T) done"
