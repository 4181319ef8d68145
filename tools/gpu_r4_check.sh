#!/bin/bash
# Round-4 last check of the committed tree: GPU suite, smoke, one config-2 bench line.
set -o pipefail
OUT=gpurun_out/${TAG:-r04zy}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2', round(d['ms_per_step'],2), d.get('parity_rel'), d['roofline'].get('frac'))" $OUT/bench_c2.json
