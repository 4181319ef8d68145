#!/bin/bash
# Round 5, run e: product = row-quad producers + edge-folded consumers; int8/parity tests on
# the product, ozcheck and ozovl, ingest tests; pass_bench product / edge0 / ovl (+ stamps);
# config-2 bench lines alternated.
set -o pipefail
OUT=gpurun_out/${TAG:-r05e}; mkdir -p $OUT; export TMPDIR=/tmp
K="ozaki or config2 or shapes or standardized or config1 or robust or wave_split or edge_strip"
for v in base ozcheck ozovl; do
  if [ $v = base ]; then L=""; else L=var/libdlsa_hip_$v.so; fi
  echo "[r5e] $(date +%T) pytest $v"
  DLSA_LIB=$L timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "$K" > $OUT/pytest_$v.log 2>&1; rc=$?
  echo "$v rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; grep FAILED $OUT/pytest_$v.log | head -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
echo "[r5e] $(date +%T) pytest ingest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -v --timeout 240 --timeout-method thread > $OUT/pytest_ingest.log 2>&1; rc=$?
echo "ingest rc=$rc: $(tail -1 $OUT/pytest_ingest.log)"; grep FAILED $OUT/pytest_ingest.log | head -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[r5e] $(date +%T) pass_bench"
timeout -k 10 600 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --rounds 3 --libs base,ozedge0,ozovl,ozprof,ozovlprof > $OUT/pass_bench.jsonl 2> $OUT/pass_bench.err || exit $?
cat $OUT/pass_bench.jsonl
for i in 1 2; do
  for v in base ozedge0 ozovl; do
    if [ $v = base ]; then L=""; else L=var/libdlsa_hip_$v.so; fi
    DLSA_LIB=$L timeout -k 10 300 python -u bench.py --config 2 --steps 3 --no-cpu-baseline --no-fp64-step > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" $OUT/bench_${v}_$i.json $v
  done
done
echo "[r5e] $(date +%T) done"
