#!/bin/bash
# Round-4 first session: X-stream cache policy (nt) A/B and warm-level sweep at config 2.
set -o pipefail
OUT=gpurun_out/r04a
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_bench_ab.sh r04a nt 2 2 || exit $?
for LV in "0.0625" "0.0625,0.25" "0.03125,0.125" "0.125"; do
  DLSA_LEVELS=$LV timeout -k 10 300 python -u bench.py --config 2 --steps 4 --no-cpu-baseline \
      > $OUT/lv_$LV.json 2> $OUT/lv_$LV.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('levels', sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'])" $OUT/lv_$LV.json $LV
done
