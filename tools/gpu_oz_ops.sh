#!/bin/bash
# Exact-pass operand / digit-batch A/B: int8 GPU tests on the product build, then
# tools/pass_bench.py over the variants (one process, interleaved rounds).
set -o pipefail
OUT=gpurun_out/${TAG:-ozops}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "ozaki or heavy or config2" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; grep -E "FAILED" $OUT/pytest.log | head
[ $rc -eq 0 ] || exit $rc
for v in $VARIANT_TEST; do  # the int8 tests on a variant build
  DLSA_LIB=tools/_variants/libdlsa_hip_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "ozaki or config2" > $OUT/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --rounds 3 \
    --libs ${LIBS:-base,ozold,ozs1,ozbt,ozdb,ozprof,ozs1prof,ozoldprof} > $OUT/pass_bench.jsonl 2> $OUT/pass_bench.err
rc=$?; cat $OUT/pass_bench.jsonl; tail -3 $OUT/pass_bench.err; [ $rc -eq 0 ] || exit $rc
# config-2 bench, product vs BENCH_ALT (a variant .so), alternated
if [ -n "$BENCH_ALT" ]; then
  for i in 1 2; do
    for v in base $BENCH_ALT; do
      if [ $v = base ]; then L=""; else L=tools/_variants/libdlsa_hip_$v.so; fi
      DLSA_LIB=$L timeout -k 10 300 python -u bench.py --config 2 --steps 3 --no-cpu-baseline --no-parity > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" $OUT/bench_${v}_$i.json $v
    done
  done
fi
