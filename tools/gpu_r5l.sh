#!/bin/bash
# Round 5, run l: exact pass on the int8 cores only with fresh max|z| records
# (polish / stale partitions -> fp64): int8 + robustness tests, config 2 bench.
set -o pipefail
OUT=gpurun_out/${TAG:-r05l}; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)), 3) for k, v in d['kernels'].items()})" "$@"; }
echo "[r5l] $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --config 2 --steps 3 --no-cpu-baseline --no-fp64-step > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
summ $OUT/bench_c2.json c2
timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --steps 10 --no-cpu-baseline --no-fp64-step > $OUT/share8.json 2> $OUT/share8.err || exit $?
summ $OUT/share8.json share8
echo "[r5l] $(date +%T) done"
