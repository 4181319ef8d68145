#!/bin/bash
# Wide-path check: wide / OLS / concurrency GPU tests, config-5 bench, kernel trace of
# config 5 (r04j: the two-lane trial; r04k on: left-looking panel Newton).  TAG= names the run.
set -o pipefail
OUT=gpurun_out/${TAG:-r04k}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "wide or config5 or p500 or P500 or concurrent or thread or ols" > $OUT/pytest_wide.log 2>&1; rc=$?
tail -3 $OUT/pytest_wide.log; grep -E "FAILED|Error" $OUT/pytest_wide.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for L in 1; do
  timeout -k 10 400 python -u bench.py --config 5 --steps 4 --no-cpu-baseline > $OUT/bench_c5_$L.json 2> $OUT/bench_c5_$L.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5', round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v,2) for k, v in d['stages_ms_per_step'].items()}, {k: round(v.get('avg_launch_ms', v.get('ms_per_step',0)), 3) for k, v in d['kernels'].items()})" $OUT/bench_c5_$L.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $OUT/prof.json 2> $OUT/prof.err || exit $?
echo done
