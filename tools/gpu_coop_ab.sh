#!/bin/bash
# bf16 pass A/B (product vs a variant build in tools/_variants, name $1) on the
# parity suite, pass timings and config-2 bench.  Usage: bash tools/gpu_coop_ab.sh <variant> <tag>
set -o pipefail
V=$1
TAG=${2:-coopab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[ab] $(date +%T) pytest" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "[ab] $(date +%T) pass A/B" &&
timeout -k 10 300 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --rounds 5 \
    --libs base,$V > "$OUT/ab_p100.jsonl" 2> "$OUT/ab_p100.err" && cat "$OUT/ab_p100.jsonl" || exit $?
for lib in base $V base $V; do
  L=""; [ $lib = $V ] && L=tools/_variants/libdlsa_hip_$V.so
  DLSA_LIB=$L timeout -k 10 600 python -u bench.py --config 2 --steps 6 --no-cpu-baseline --no-parity > "$OUT/bench_c2_$lib.json" 2> "$OUT/bench_c2_$lib.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" "$OUT/bench_c2_$lib.json" "$lib"
done
echo "[ab] $(date +%T) done"
