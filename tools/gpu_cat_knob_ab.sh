#!/bin/bash
# Categorical-path knob A/B at config 3 (r04n: warm-start levels; r04o: DLSA_CAT_MIXED
# approximate passes): categorical GPU tests with the knob on, then bench.py alternated.
set -o pipefail
OUT=gpurun_out/${TAG:-r04o}; mkdir -p $OUT; export TMPDIR=/tmp
DLSA_CAT_MIXED=1 timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "categorical or config3" > $OUT/pytest_cat_ws.log 2>&1; rc=$?
tail -3 $OUT/pytest_cat_ws.log; grep -E "FAILED" $OUT/pytest_cat_ws.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for arm in off mixed; do
    E="DLSA_AB_NONE=1"
    [ $arm = mixed ] && E="DLSA_CAT_MIXED=1"
    env $E timeout -k 10 400 python -u bench.py --config 3 --steps 4 --no-cpu-baseline > $OUT/bench_c3_${arm}_$i.json 2> $OUT/bench_c3_${arm}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v,2) for k, v in d['stages_ms_per_step'].items()})" $OUT/bench_c3_${arm}_$i.json "c3 $arm"
  done
done
