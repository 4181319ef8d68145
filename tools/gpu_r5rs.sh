#!/bin/bash
# Round 5, run rs: Newton solve, rsq refinement steps in the diagonal factor (2 / 1 / 0): config 3
# and the N=8 share of config 2 (newton_solve ms per step and parity).
set -o pipefail
OUT=gpurun_out/${TAG:-r05rs}; mkdir -p $OUT
run() {  # label lib bench-args...
  local lab=$1 lib=$2; shift 2
  DLSA_LIB=$lib timeout -k 10 200 python -u bench.py "$@" --no-cpu-baseline > $OUT/tmp.json 2>> $OUT/err.log || return $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels'].get('newton_solve',{}); print(json.dumps({'variant': sys.argv[2], 'ms_per_step': round(d['ms_per_step'],2), 'newton_ms_per_step': round(k.get('ms_per_step', 0) or 0, 3), 'newton': d['newton'].get('iterations'), 'parity_rel': d.get('parity_rel')}))" $OUT/tmp.json "$lab" | tee -a $OUT/sweep.jsonl
}
for r in 1 2; do
  for v in base:dlsa_amd/libdlsa_hip.so rsq1:var/libdlsa_hip_solversq1.so rsq0:var/libdlsa_hip_solversq0.so; do
    run "c3_${v%%:*}" "${v#*:}" --config 3 --steps 4 || exit $?
    run "s8_${v%%:*}" "${v#*:}" --n 12500000 --partitions 128 --steps 10 || exit $?
  done
done
