#!/bin/bash
# Round 5, first run: int8 exact-pass tests on the product (padding-feature race
# fixed) and on the round-4 producer-DMA variant (tools/patches/oz_producer_dma.patch,
# DLSA_OZ_SCHED 3) rebuilt with the fix; then a config-2 bench line.
set -o pipefail
OUT=gpurun_out/${TAG:-r05a}; mkdir -p $OUT; export TMPDIR=/tmp
for v in base ozs3fix; do
  if [ $v = base ]; then L=""; else L=var/libdlsa_hip_$v.so; fi
  echo "[r5a] $(date +%T) pytest $v"
  DLSA_LIB=$L timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "ozaki or config2" > $OUT/pytest_$v.log 2>&1; rc=$?
  echo "$v rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; grep FAILED $OUT/pytest_$v.log | head -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
echo "[r5a] $(date +%T) bench c2"
timeout -k 10 600 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['ms_per_step'],2), d.get('parity_rel'), d['roofline'].get('frac'), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" $OUT/bench_c2.json
echo "[r5a] $(date +%T) done"
