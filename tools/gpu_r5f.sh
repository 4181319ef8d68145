#!/bin/bash
# Round 5, run f: GPU suite on the product (row-quad producers, blocked Newton solves),
# int8 tests on the producer-DMA-split variants, pass_bench, config-2 and strong-share benches.
set -o pipefail
OUT=gpurun_out/${TAG:-r05f}; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r5f] $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
K="ozaki or config2 or shapes or standardized"
for v in ozpd1 ozpd2 ozpd3; do
  echo "[r5f] $(date +%T) pytest $v"
  DLSA_LIB=var/libdlsa_hip_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "$K" > $OUT/pytest_$v.log 2>&1; rc=$?
  echo "$v rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; grep FAILED $OUT/pytest_$v.log | head -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
echo "[r5f] $(date +%T) pass_bench"
timeout -k 10 600 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --rounds 3 --libs base,ozpd1,ozpd2,ozpd3,ozprof,ozpd2prof > $OUT/pass_bench.jsonl 2> $OUT/pass_bench.err || exit $?
cat $OUT/pass_bench.jsonl
for i in 1 2; do
  for v in base ozpd1 ozpd2 ozpd3; do
    if [ $v = base ]; then L=""; else L=var/libdlsa_hip_$v.so; fi
    DLSA_LIB=$L timeout -k 10 300 python -u bench.py --config 2 --steps 3 --no-cpu-baseline --no-fp64-step > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)), 3) for k, v in d['kernels'].items()})" $OUT/bench_${v}_$i.json $v
  done
  for v in base solveold; do
    if [ $v = base ]; then L=""; else L=var/libdlsa_hip_$v.so; fi
    DLSA_LIB=$L timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --steps 10 --no-cpu-baseline --no-fp64-step > $OUT/share8_${v}_$i.json 2> $OUT/share8_${v}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('share8', sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v, 3) for k, v in d['stages_ms_per_step'].items()}, {k: round(v.get('ms_per_step', 0), 3) for k, v in d['kernels'].items()})" $OUT/share8_${v}_$i.json $v
  done
done
echo "[r5f] $(date +%T) bench c3"
timeout -k 10 400 python -u bench.py --config 3 --steps 4 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c3', round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)), 3) for k, v in d['kernels'].items()})" $OUT/bench_c3.json
echo "[r5f] $(date +%T) kernel trace c3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $OUT/prof_c3.json 2> $OUT/prof_c3.err || exit $?
echo "[r5f] $(date +%T) done"
