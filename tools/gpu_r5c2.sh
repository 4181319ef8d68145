#!/bin/bash
# Round 5, run c2: config-2 chunk-size sweep on the current kernels (knobs build, DLSA_ROWS_PER_CHUNK).
set -o pipefail
OUT=gpurun_out/${TAG:-r05c2}; mkdir -p $OUT
export DLSA_LIB=var/libdlsa_hip_knobs.so
for r in 16384 8192 12288 24576 32768 16384; do
  DLSA_ROWS_PER_CHUNK=$r timeout -k 10 150 python -u bench.py --config 2 --steps 4 --warmup 2 --no-cpu-baseline > $OUT/tmp.json 2>> $OUT/err.log || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'rows_per_chunk': int(sys.argv[2]), 'ms_per_step': round(d['ms_per_step'],2), 'kernels': {k: round(v.get('avg_launch_ms',0),3) for k,v in d['kernels'].items()}, 'n_chunks': d['newton'].get('n_chunks'), 'parity_rel': d.get('parity_rel')}))" $OUT/tmp.json $r | tee -a $OUT/sweep.jsonl
done
