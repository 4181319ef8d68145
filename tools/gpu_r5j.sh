#!/bin/bash
# Round 5, run j: chunk-size A/B at the N=8 strong-scaling share of config 2
# (knobs build, DLSA_ROWS_PER_CHUNK; the product picks 4096 rows there).
set -o pipefail
OUT=gpurun_out/${TAG:-r05j}; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton']['n_chunks'], {k: round(v.get('ms_per_step', 0), 3) for k, v in d['kernels'].items()}, {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" "$@"; }
for i in 1 2; do
  for r in 4096 6144 8192 12288; do
    DLSA_LIB=var/libdlsa_hip_knobs.so DLSA_ROWS_PER_CHUNK=$r timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --steps 10 --no-cpu-baseline --no-fp64-step > $OUT/share8_r${r}_$i.json 2> $OUT/share8_r${r}_$i.err || exit $?
    summ $OUT/share8_r${r}_$i.json share8_r$r
  done
done
echo "[r5j] $(date +%T) done"
