#!/bin/bash
# Round 5, run ce: the exact-bucket categorical kernel (EX: compile-time column
# count and intercept) vs the previous pass (cathead): bit-identity across
# builds, the categorical GPU tests, config-3 A/B; then the ablations of
# gpu_r5ca.sh on the previous pass (ABL="cat16 cat1 ..."; tools/build_variants.sh).
# Needs var/libdlsa_hip_cathead.so: a copy of the in-tree library built
# before the change (cp dlsa_amd/libdlsa_hip.so var/libdlsa_hip_cathead.so).
set -o pipefail
OUT=gpurun_out/${TAG:-r05ce}; mkdir -p $OUT
PYTHONPATH=. DLSA_LIB=var/libdlsa_hip_cathead.so timeout -k 10 120 python -u tools/cat_xbuild.py $OUT/old.npz > $OUT/xb.log 2>&1 || exit $?
PYTHONPATH=. timeout -k 10 120 python -u tools/cat_xbuild.py $OUT/new.npz >> $OUT/xb.log 2>&1 || exit $?
python tools/cat_xbuild.py --compare $OUT/old.npz $OUT/new.npz | tee -a $OUT/xb.log || exit $?
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_robustness.py -k categorical > $OUT/pytest.log 2>&1 || exit $?
tail -1 $OUT/pytest.log
run() {
  DLSA_LIB=$2 timeout -k 10 200 python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline --no-parity > $OUT/tmp.json 2>> $OUT/err.log || return $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels']['cat_pass_kernel']; print(json.dumps({'variant': sys.argv[2], 'ms_per_step': round(d['ms_per_step'],2), 'launches': k['launches_per_step'], 'cat_ms_per_step': round(k['ms_per_step'],3), 'cat_avg_launch_ms': round(k['avg_launch_ms'],3)}))" $OUT/tmp.json "$1" | tee -a $OUT/sweep.jsonl
}
for r in 1 2; do
  run ${NEWTAG:-exact} dlsa_amd/libdlsa_hip.so || exit $?
  run head var/libdlsa_hip_cathead.so || exit $?
done
[ -n "$ABL" ] && for v in $ABL; do run $v var/libdlsa_hip_$v.so || exit $?; done; true
