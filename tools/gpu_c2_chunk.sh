#!/bin/bash
# Config-2 rows-per-chunk A/B, alternated: the current rule vs the old n/8192 (12207 rows).
set -o pipefail
OUT=gpurun_out/${1:-c2chunk}; mkdir -p $OUT; export TMPDIR=/tmp
for r in "" 12207 "" 12207 "" 12207; do
  env ${r:+DLSA_ROWS_PER_CHUNK=$r} timeout -k 10 300 python -u bench.py --steps 4 --no-cpu-baseline --no-parity > $OUT/c2.json 2> $OUT/c2.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2 rpc', sys.argv[2], round(d['ms_per_step'],2), d['newton']['n_chunks'], {k: round(v.get('ms_per_step', 0), 3) for k, v in d['kernels'].items()})" $OUT/c2.json "${r:-auto}"
done
