#!/bin/bash
# Parity suite + config 2 / config 4 / strong-share benches with the current chunk rule.
set -o pipefail
OUT=gpurun_out/${1:-verify}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -1 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --scaling strong --n 12500000 --partitions 128 --steps 8 --no-cpu-baseline > $OUT/strong.json 2> $OUT/strong.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('strong', round(d['ms_per_step'],2), d['newton']['n_chunks'], d.get('parity_rel'), d['roofline']['frac'])" $OUT/strong.json
  timeout -k 10 300 python -u bench.py --steps 4 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2', round(d['ms_per_step'],2), d['newton']['n_chunks'], d.get('parity_rel'), d['roofline']['frac'])" $OUT/c2.json
  timeout -k 10 300 python -u bench.py --config 4 --steps 4 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c4', round(d['ms_per_step'],2), d['newton']['n_chunks'], d.get('parity_rel'), d['roofline']['frac'])" $OUT/c4.json
done
