#!/bin/bash
# Round 5, run wr: wide row pass rows per wave and step (U = 2 / 4 / 8), config 5.
set -o pipefail
OUT=gpurun_out/${TAG:-r05wr2}; mkdir -p $OUT
run() {
  DLSA_LIB=$2 timeout -k 10 200 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $OUT/tmp.json 2>> $OUT/err.log || return $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'variant': sys.argv[2], 'ms_per_step': round(d['ms_per_step'],2), 'row_ms': round(d['kernels']['wide_row_kernel'].get('ms_per_step',0),3), 'gram_ms': round([v for k,v in d['kernels'].items() if 'oz_gram' in k][0].get('avg_launch_ms',0),3)}))" $OUT/tmp.json "$1" | tee -a $OUT/sweep.jsonl
}
for r in 1 2; do
  run u4 dlsa_amd/libdlsa_hip.so || exit $?
  run u2 var/libdlsa_hip_wrow2.so || exit $?
done
