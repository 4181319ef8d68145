#!/bin/bash
# Round 5, run g: GPU suite (streaming presence pass, OLS row-sequential row phase +
# column swap), config 3 / config 4 benches with OLS A/B variants, config-2 kernel
# traces of the product and the cmabl variant (first full bf16 pass A/B), share8.
set -o pipefail
OUT=gpurun_out/${TAG:-r05g}; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)), 3) for k, v in d['kernels'].items()}, {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" "$@"; }
echo "[r5g] $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[r5g] $(date +%T) bench c3"
timeout -k 10 400 python -u bench.py --config 3 --steps 4 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
summ $OUT/bench_c3.json c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $OUT/prof_c3.json 2> $OUT/prof_c3.err || exit $?
for i in 1 2; do
  for v in base olsold olsnoswap; do
    if [ $v = base ]; then L=""; else L=var/libdlsa_hip_$v.so; fi
    DLSA_LIB=$L timeout -k 10 300 python -u bench.py --config 4 --steps 5 --no-cpu-baseline > $OUT/bench_c4_${v}_$i.json 2> $OUT/bench_c4_${v}_$i.err || exit $?
    summ $OUT/bench_c4_${v}_$i.json c4_$v
  done
done
echo "[r5g] $(date +%T) c2 traces"
for v in base cmabl; do
  if [ $v = base ]; then L=""; else L=var/libdlsa_hip_$v.so; fi
  DLSA_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2_$v -o run -- python3 bench.py --config 2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/prof_c2_$v.json 2> $OUT/prof_c2_$v.err || exit $?
done
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --steps 10 --no-cpu-baseline --no-fp64-step > $OUT/share8_$i.json 2> $OUT/share8_$i.err || exit $?
  summ $OUT/share8_$i.json share8
done
echo "[r5g] $(date +%T) done"
