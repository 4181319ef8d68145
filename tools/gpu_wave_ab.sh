#!/bin/bash
# Exact-pass A/B (product vs a variant build tools/_variants/libdlsa_hip_$1.so):
# parity suite, pass timings at P = 100 / 64 and the config-2 / config-4 benches
# of both builds.  Usage: bash tools/gpu_wave_ab.sh <variant> <tag>
set -o pipefail
V=$1
TAG=${2:-waveab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[ab] $(date +%T) pytest" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo "[ab] $(date +%T) exact pass A/B" &&
for pp in 100 64; do
  timeout -k 10 300 python -u tools/pass_bench.py --n 25000000 --p $pp --K 256 --hessian fp64 --rounds 5 \
      --libs base,$V > "$OUT/ab_p$pp.jsonl" 2> "$OUT/ab_p$pp.err" && cat "$OUT/ab_p$pp.jsonl" || exit $?
done
for c in 2 4; do
  for lib in base $V base $V; do
    L=""; [ $lib = $V ] && L=tools/_variants/libdlsa_hip_$V.so
    DLSA_LIB=$L timeout -k 10 600 python -u bench.py --config $c --steps 6 --no-cpu-baseline > "$OUT/bench_c${c}_$lib.json" 2> "$OUT/bench_c${c}_$lib.err" || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" "$OUT/bench_c${c}_$lib.json" "c$c $lib"
  done
done
echo "[ab] $(date +%T) done"
