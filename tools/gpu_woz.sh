#!/bin/bash
# Wide int8 exact Gram: its GPU tests, the wide parity tests, config-5 A/B.
set -o pipefail
TAG=${1:-woz}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[woz] $(date +%T) ozaki tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ozaki.py -m gpu -v --timeout 120 \
    --timeout-method thread -x -k wide > "$OUT/pytest_ozaki.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_ozaki.log"; grep -E "^E .*(assert|Error)|FAILED|^E  " "$OUT/pytest_ozaki.log" | head -20
[ $rc -eq 0 ] || exit $rc
echo "[woz] $(date +%T) wide parity"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
    -k "wide or p500 or config5 or maxiter" > "$OUT/pytest_wide.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_wide.log"; grep -E "^E .*(assert|Error)|FAILED" "$OUT/pytest_wide.log" | head -20
[ $rc -eq 0 ] || exit $rc
for k in default 0; do
  echo "[woz] $(date +%T) bench c5 DLSA_OZ=$k"
  if [ $k = default ]; then unset DLSA_OZ; else export DLSA_OZ=$k; fi
  timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline > "$OUT/bench_c5_$k.json" 2> "$OUT/bench_c5_$k.err" || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {a: round(b.get('avg_launch_ms', b.get('ms_per_step', 0)),3) for a,b in d['kernels'].items()}, d['stages_ms_per_step'])" "$OUT/bench_c5_$k.json" $k
done
unset DLSA_OZ
echo "[woz] $(date +%T) rocprof c5"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run -- \
    python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > "$OUT/bench_prof_c5.json" 2> "$OUT/prof_c5.err"
echo "[woz] $(date +%T) done"
