#!/bin/bash
# Round 5, run d: row-quad producers + producer-issued DMA (DLSA_OZ_SCHED 3/4/5):
# int8 tests, pass_bench, config-2 bench lines.
set -o pipefail
OUT=gpurun_out/${TAG:-r05d}; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r5d] $(date +%T) pytest ingest (device data_info)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py -v --timeout 240 --timeout-method thread > $OUT/pytest_ingest.log 2>&1; rc=$?
echo "ingest rc=$rc: $(tail -1 $OUT/pytest_ingest.log)"; grep FAILED $OUT/pytest_ingest.log | head -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in ozr4s3 ozr4s4 ozr4s5; do
  echo "[r5d] $(date +%T) pytest $v"
  DLSA_LIB=var/libdlsa_hip_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "ozaki or config2 or shapes or standardized or config1" > $OUT/pytest_$v.log 2>&1; rc=$?
  echo "$v rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; grep FAILED $OUT/pytest_$v.log | head -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
echo "[r5d] $(date +%T) pass_bench"
timeout -k 10 600 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --rounds 3 --libs base,ozr4,ozr4s3,ozr4s4,ozr4s5,ozr4s4prof > $OUT/pass_bench.jsonl 2> $OUT/pass_bench.err || exit $?
cat $OUT/pass_bench.jsonl
for i in 1 2; do
  for v in ozr4 ozr4s3 ozr4s4 ozr4s5; do
    L=var/libdlsa_hip_$v.so
    DLSA_LIB=$L timeout -k 10 300 python -u bench.py --config 2 --steps 3 --no-cpu-baseline --no-fp64-step > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" $OUT/bench_${v}_$i.json $v
  done
done
echo "[r5d] $(date +%T) done"
