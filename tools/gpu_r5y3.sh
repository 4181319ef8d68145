#!/bin/bash
# Round 5, run y3: pinned upload arena -- GPU suite, config-5 runtime trace (4 steps: does any fit's
# first command still wait?), config 2 and 5 bench lines.
set -o pipefail
OUT=gpurun_out/${TAG:-r05y3}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 rocprofv3 --runtime-trace --stats -d $OUT/rt_c5 -o run -- python3 bench.py --config 5 --steps 4 --warmup 1 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/rt_c5.json 2> $OUT/rt_c5.err || exit $?
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config 5 --steps 4 --no-cpu-baseline > $OUT/bench_c5_$r.json 2> $OUT/bench_c5_$r.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5', round(d['ms_per_step'],2), {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" $OUT/bench_c5_$r.json
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2', round(d['ms_per_step'],2), {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" $OUT/bench_c2.json
