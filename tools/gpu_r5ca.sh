#!/bin/bash
# Round 5, run ca: categorical pass ablations on the current pass (per-launch
# time only; an ablated pass computes a wrong Hessian, so the fit's pass count
# may move): 16 no slab-epilogue lookups, 1 no numeric x dummy adds, 8 no
# numeric register block, 7 no histogram adds at all.
set -o pipefail
OUT=gpurun_out/${TAG:-r05ca}; mkdir -p $OUT
run() {
  DLSA_LIB=$2 timeout -k 10 200 python -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $OUT/tmp.json 2>> $OUT/err.log || return $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']['cat_pass_kernel']; print(json.dumps({'variant': sys.argv[2], 'ms_per_step': round(d['ms_per_step'],2), 'launches': k['launches_per_step'], 'cat_ms_per_step': round(k['ms_per_step'],3), 'cat_avg_launch_ms': round(k['avg_launch_ms'],3)}))" $OUT/tmp.json "$1" | tee -a $OUT/sweep.jsonl
}
run product dlsa_amd/libdlsa_hip.so || exit $?
for v in cat16 cat1 cat8 cat7; do run $v var/libdlsa_hip_$v.so || exit $?; done
