#!/bin/bash
# Exact-pass edge strip A/B: product (last tile row as v_mfma_f64_4x4x4_4b
# sub-blocks) vs the DLSA_WAVE_STRIP=0 build, pass timings, the config-2 bench
# of both builds and a kernel trace of the product (gaps between launches).
# Usage: bash tools/gpu_strip.sh <tag>
set -o pipefail
TAG=${1:-strip}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[strip] $(date +%T) A/B exact pass" &&
timeout -k 10 300 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --hessian fp64 --rounds 5 \
    --libs base,strip0 > "$OUT/ab_p100.jsonl" 2> "$OUT/ab_p100.err" && cat "$OUT/ab_p100.jsonl" || exit $?
for lib in base strip0 base strip0; do
  L=""; [ $lib = strip0 ] && L=tools/_variants/libdlsa_hip_strip0.so
  DLSA_LIB=$L timeout -k 10 600 python -u bench.py --config 2 --steps 6 --no-cpu-baseline --no-parity > "$OUT/bench_c2_$lib.json" 2> "$OUT/bench_c2_$lib.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d['stages_ms_per_step'], {k: round(v.get('ms_per_step', 0), 2) for k, v in d['kernels'].items()})" "$OUT/bench_c2_$lib.json" "$lib"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_c2" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/trace_c2.json" 2> "$OUT/trace_c2.err" &&
echo "[strip] $(date +%T) done"
