#!/bin/bash
# Config-3 bench with the current chunk rule and with the old 8192-chunk rows.
set -o pipefail
OUT=gpurun_out/${1:-c3check}; mkdir -p $OUT; export TMPDIR=/tmp
for r in "" 1831 "" 1831; do
  env ${r:+DLSA_ROWS_PER_CHUNK=$r} timeout -k 10 300 python -u bench.py --config 3 --steps 6 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c3 rpc', sys.argv[2], round(d['ms_per_step'],2), d['newton']['n_chunks'], d.get('parity_rel'), {k: round(v.get('ms_per_step', 0), 3) for k, v in d['kernels'].items()})" $OUT/c3.json "${r:-auto}"
done
