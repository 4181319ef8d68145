#!/bin/bash
# Round 5, run fw: wide fused bf16 pass with 8 waves per workgroup (two per SIMD, 4 rows and
# 33 tiles each) against 4 (one per SIMD): wide GPU tests on the variant, config-5 A/B.
set -o pipefail
OUT=gpurun_out/${TAG:-r05fw}; mkdir -p $OUT
DLSA_LIB=var/libdlsa_hip_wfw8.so timeout -k 10 600 python -u -m pytest tests -m gpu -k "wide or Wide" -x -q --timeout 240 --timeout-method thread > $OUT/pytest_wide_fw8.log 2>&1 || { tail -30 $OUT/pytest_wide_fw8.log; exit 1; }
tail -1 $OUT/pytest_wide_fw8.log
run() {
  DLSA_LIB=$2 timeout -k 10 200 python -u bench.py --config 5 --steps 4 --warmup 1 --no-cpu-baseline > $OUT/tmp.json 2>> $OUT/err.log || return $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']['wide_fused_bf16_kernel']; print(json.dumps({'variant': sys.argv[2], 'ms_per_step': round(d['ms_per_step'],2), 'fused_avg_ms': round(k['avg_launch_ms'],3), 'fused_GBps': round(k['GBps']), 'fit': round(d['stages_ms_per_step']['fit'],2), 'parity_rel': d.get('parity_rel'), 'iters': d['newton'].get('iterations')}))" $OUT/tmp.json "$1" | tee -a $OUT/sweep.jsonl
}
for r in 1 2; do
  run fw4 dlsa_amd/libdlsa_hip.so || exit $?
  run fw8 var/libdlsa_hip_wfw8.so || exit $?
done
