#!/bin/bash
# Config-5 runtime knob sweep (warm-start level tolerance / levels), bench.py alternated.
set -o pipefail
OUT=gpurun_out/${TAG:-r04p}; mkdir -p $OUT; export TMPDIR=/tmp
for i in 1 2; do
  for arm in base lt2 lt3 lv1; do
    E="DLSA_AB_NONE=1"
    [ $arm = lt2 ] && E="DLSA_LEVEL_TOL=0.2"
    [ $arm = lt3 ] && E="DLSA_LEVEL_TOL=0.3"
    [ $arm = lv1 ] && E="DLSA_LEVELS=0.0625"
    env $E timeout -k 10 400 python -u bench.py --config 5 --steps 4 --no-cpu-baseline > $OUT/bench_c5_${arm}_$i.json 2> $OUT/bench_c5_${arm}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], round(d['stages_ms_per_step']['fit'],2))" $OUT/bench_c5_${arm}_$i.json "c5 $arm"
  done
done
