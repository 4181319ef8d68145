#!/bin/bash
# Exact-pass row-phase geometry A/B at P <= 64 (product vs tools/_variants/libdlsa_hip_$1.so):
# the variant's GPU parity suite, the p = 64 fp64 pass and config 4 (OLS) alternated.
# Usage: bash tools/gpu_lpr_ab.sh "<variant> [<variant> ...]" <tag>
# (r02as / r02at ran builds with the since-removed DLSA_WAVE_LPR4_NT, DLSA_WAVE_LPR16_NT
# and DLSA_WAVE_MINW_SMALL defines; r02at's lpr16o5 is now the OLS default)
set -o pipefail
VS=$1
TAG=${2:-lprab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for V in $VS; do
  echo "[ab] $(date +%T) pytest ($V)" &&
  DLSA_LIB=tools/_variants/libdlsa_hip_$V.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
      --timeout 240 --timeout-method thread > "$OUT/pytest_gpu_$V.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest_gpu_$V.log"; [ $rc -eq 0 ] || exit $rc
done
echo "[ab] $(date +%T) p=64 exact pass A/B" &&
timeout -k 10 300 python -u tools/pass_bench.py --n 25000000 --p 64 --K 256 --hessian fp64 --rounds 6 \
    --libs base,${VS// /,} > "$OUT/ab_p64.jsonl" 2> "$OUT/ab_p64.err" && cat "$OUT/ab_p64.jsonl" || exit $?
for i in 1 2 3; do
  for lib in base $VS; do
    L=""; [ $lib != base ] && L=tools/_variants/libdlsa_hip_$lib.so
    DLSA_LIB=$L timeout -k 10 600 python -u bench.py --config 4 --steps 8 --no-cpu-baseline > "$OUT/bench_c4_${lib}_$i.json" 2> "$OUT/bench_c4_${lib}_$i.err" || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" "$OUT/bench_c4_${lib}_$i.json" "c4 $lib $i"
  done
done
echo "[ab] $(date +%T) done"
