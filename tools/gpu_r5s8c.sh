#!/bin/bash
# Round 5, run s8c: chunk size at the N=8 per-rank share of config 2 (knobs build).
set -o pipefail
OUT=gpurun_out/${TAG:-r05s8c}; mkdir -p $OUT
export DLSA_LIB=var/libdlsa_hip_knobs.so
for r in 1 2; do
  for rpc in 6144 8192 12288 16384 4096; do
    DLSA_ROWS_PER_CHUNK=$rpc timeout -k 10 150 python -u bench.py --n 12500000 --partitions 128 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/tmp.json 2>> $OUT/err.log || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'rows_per_chunk': int(sys.argv[2]), 'ms_per_step': round(d['ms_per_step'],3), 'kernels': {k: round(v.get('avg_launch_ms',0) or 0,3) for k,v in d['kernels'].items()}, 'parity_rel': d.get('parity_rel')}))" $OUT/tmp.json $rpc | tee -a $OUT/sweep.jsonl
  done
done
