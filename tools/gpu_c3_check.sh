#!/bin/bash
# Config-3 check: categorical GPU tests, two config-3 benches, a config-3 kernel trace.
set -o pipefail
OUT=gpurun_out/${TAG:-c3check}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "categorical or config3 or cat_" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; grep -E "FAILED" $OUT/pytest.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --config 3 --steps 4 --no-cpu-baseline > $OUT/bench_c3_$i.json 2> $OUT/bench_c3_$i.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c3', round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v,2) for k, v in d['stages_ms_per_step'].items()})" $OUT/bench_c3_$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $OUT/prof.json 2> $OUT/prof.err || exit $?
echo done
