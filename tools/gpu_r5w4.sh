#!/bin/bash
# Round 5, run w4: warm-start level row floor (rows per parameter) x schedule, config 5 (knobs build).
set -o pipefail
OUT=gpurun_out/${TAG:-r05w4}; mkdir -p $OUT
export DLSA_LIB=var/libdlsa_hip_knobs.so
for rpp in 8 16 32 64; do
  for lv in "0.0625,0.25" "0.0625"; do
    DLSA_LEVEL_ROWS_PER_P=$rpp DLSA_LEVELS="$lv" DLSA_LEVEL_TOL=0.1 timeout -k 10 150 python -u bench.py --config 5 \
        --steps 3 --warmup 1 --no-cpu-baseline > $OUT/tmp.json 2>> $OUT/err.log || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'rows_per_p': int(sys.argv[2]), 'levels': sys.argv[3], 'ms_per_step': round(d['ms_per_step'],2), 'fit': round(d['stages_ms_per_step']['fit'],2), 'newton': d['newton'], 'parity_rel': d.get('parity_rel')}))" $OUT/tmp.json $rpp "$lv" | tee -a $OUT/sweep.jsonl
  done
done
