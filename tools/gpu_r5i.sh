#!/bin/bash
# Round 5, run i: new robustness / polish tests + full GPU suite (EMAX overflow
# chunks fail visibly), Newton solve phase profile at configs 3 and 2-share.
set -o pipefail
OUT=gpurun_out/${TAG:-r05i}; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r5i] $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu.log; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[r5i] $(date +%T) solve profile"
DLSA_LIB=var/libdlsa_hip_solveprof.so timeout -k 10 300 python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $OUT/solveprof_c3.json 2> $OUT/solveprof_c3.err || exit $?
grep -h "solve-profile" $OUT/solveprof_c3.json $OUT/solveprof_c3.err | head -12
DLSA_LIB=var/libdlsa_hip_solveprof.so timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/solveprof_s8.json 2> $OUT/solveprof_s8.err || exit $?
grep -h "solve-profile" $OUT/solveprof_s8.json $OUT/solveprof_s8.err | head -12
echo "[r5i] $(date +%T) done"
echo "[r5i] $(date +%T) benches"
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)), 3) for k, v in d['kernels'].items()}, {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" "$@"; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --steps 10 --no-cpu-baseline --no-fp64-step > $OUT/share8_$i.json 2> $OUT/share8_$i.err || exit $?
  summ $OUT/share8_$i.json share8
  timeout -k 10 400 python -u bench.py --config 3 --steps 4 --no-cpu-baseline > $OUT/bench_c3_$i.json 2> $OUT/bench_c3_$i.err || exit $?
  summ $OUT/bench_c3_$i.json c3
  timeout -k 10 300 python -u bench.py --config 2 --steps 3 --no-cpu-baseline --no-fp64-step > $OUT/bench_c2_$i.json 2> $OUT/bench_c2_$i.err || exit $?
  summ $OUT/bench_c2_$i.json c2
done
echo "[r5i] $(date +%T) done2"
