#!/bin/bash
# Round 5, run ok2: OLS stream kernel -- k-steps in flight (KS 2 / 4 / 8: occupancy 4 / 3 / 2 waves
# per SIMD) and chunk size, config 4.
set -o pipefail
OUT=gpurun_out/${TAG:-r05ok2}; mkdir -p $OUT
run() {  # label lib [rows_per_chunk]
  local lab=$1 lib=$2 rpc=$3
  DLSA_LIB=$lib DLSA_ROWS_PER_CHUNK=$rpc timeout -k 10 150 python -u bench.py --config 4 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/tmp.json 2>> $OUT/err.log || return $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'variant': sys.argv[2], 'ms_per_step': round(d['ms_per_step'],2), 'pass_ms': [round(v.get('avg_launch_ms',0),3) for k,v in d['kernels'].items()][0], 'parity_rel': d.get('parity_rel')}))" $OUT/tmp.json "$lab" | tee -a $OUT/sweep.jsonl
}
for r in 1 2; do
  run base dlsa_amd/libdlsa_hip.so "" || exit $?
  run ks8 var/libdlsa_hip_olsks8.so "" || exit $?
  run ks12 var/libdlsa_hip_olsks12.so "" || exit $?
  run ks16 var/libdlsa_hip_olsks16.so "" || exit $?
done
