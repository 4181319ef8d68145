#!/bin/bash
# Round 5, run k: GPU suite (chunk floor 6144, trisolve address selects), and the
# fp32-MFMA approximate Hessian (hessian=mixed_f32) against bf16 at config 2 / share8.
set -o pipefail
OUT=gpurun_out/${TAG:-r05k}; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)), 3) for k, v in d['kernels'].items()}, {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" "$@"; }
echo "[r5k] $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for h in mixed mixed_f32; do
    timeout -k 10 300 python -u bench.py --config 2 --steps 3 --hessian $h --no-cpu-baseline --no-fp64-step > $OUT/bench_c2_${h}_$i.json 2> $OUT/bench_c2_${h}_$i.err || exit $?
    summ $OUT/bench_c2_${h}_$i.json c2_$h
    timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --steps 10 --hessian $h --no-cpu-baseline --no-fp64-step > $OUT/share8_${h}_$i.json 2> $OUT/share8_${h}_$i.err || exit $?
    summ $OUT/share8_${h}_$i.json share8_$h
  done
done
echo "[r5k] $(date +%T) done"
