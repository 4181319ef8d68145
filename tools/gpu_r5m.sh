#!/bin/bash
# Round 5, run m: wide Newton solve with rsq + reciprocal diagonal (product) vs IEEE
# sqrt/div (widercp0) at config 5; wide GPU tests on the product; categorical chunking
# by total rows / 512 (product) vs 512 / K chunks per partition (catper) at config 3.
set -o pipefail
OUT=gpurun_out/${TAG:-r05m}; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)), 3) for k, v in d['kernels'].items()}, {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" "$@"; }
echo "[r5m] $(date +%T) pytest wide"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "wide or config5 or maxiter or categorical or config3" > $OUT/pytest_wide.log 2>&1
rc=$?; tail -1 $OUT/pytest_wide.log; grep -E "FAILED" $OUT/pytest_wide.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for v in base widercp0; do
    if [ $v = base ]; then L=""; else L=var/libdlsa_hip_$v.so; fi
    DLSA_LIB=$L timeout -k 10 400 python -u bench.py --config 5 --steps 3 --no-cpu-baseline --no-fp64-step > $OUT/bench_c5_${v}_$i.json 2> $OUT/bench_c5_${v}_$i.err || exit $?
    summ $OUT/bench_c5_${v}_$i.json c5_$v
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o run -- python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/prof_c5.json 2> $OUT/prof_c5.err || exit $?
for i in 1 2; do
  for v in base catper; do
    if [ $v = base ]; then L=""; else L=var/libdlsa_hip_$v.so; fi
    DLSA_LIB=$L timeout -k 10 400 python -u bench.py --config 3 --steps 4 --no-cpu-baseline > $OUT/bench_c3_${v}_$i.json 2> $OUT/bench_c3_${v}_$i.err || exit $?
    summ $OUT/bench_c3_${v}_$i.json c3_$v
  done
done
echo "[r5m] $(date +%T) done"
