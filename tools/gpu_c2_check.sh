#!/bin/bash
# Config-2 check: int8 / exponent GPU tests, two config-2 benches, a config-2 kernel trace.
set -o pipefail
OUT=gpurun_out/${TAG:-c2check}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "ozaki or config2 or heavy" > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; grep -E "FAILED" $OUT/pytest.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --config 2 --steps 4 --no-cpu-baseline > $OUT/bench_c2_$i.json 2> $OUT/bench_c2_$i.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2', round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" $OUT/bench_c2_$i.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --config 2 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $OUT/prof.json 2> $OUT/prof.err || exit $?
echo done
