#!/bin/bash
# Chunk-size A/B at the config-2 strong-scaling share (n = 1.25e7, K = 128) and at config 2.
set -o pipefail
OUT=gpurun_out/${1:-chunkab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in "" 3072 6144 12288 ""; do
  env ${r:+DLSA_ROWS_PER_CHUNK=$r} timeout -k 10 300 python -u bench.py --scaling strong --n 12500000 --partitions 128 --steps 8 --no-cpu-baseline --no-parity > "$OUT/s.json" 2> "$OUT/s.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('strong rpc', sys.argv[2], round(d['ms_per_step'],2), d['newton']['n_chunks'], {k: round(v.get('ms_per_step', 0), 3) for k, v in d['kernels'].items()}, round(d['stages_ms_per_step']['fit_native'],2))" "$OUT/s.json" "${r:-auto}"
done
for r in "" 16384; do
  env ${r:+DLSA_ROWS_PER_CHUNK=$r} timeout -k 10 300 python -u bench.py --steps 4 --no-cpu-baseline --no-parity > "$OUT/c2.json" 2> "$OUT/c2.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c2 rpc', sys.argv[2], round(d['ms_per_step'],2), d['newton']['n_chunks'], {k: round(v.get('ms_per_step', 0), 3) for k, v in d['kernels'].items()})" "$OUT/c2.json" "${r:-auto}"
done
