#!/bin/bash
# r04h: OLS pass A/B -- product (3 ring slots, one barrier per full block) vs
# 2 slots, vs two barriers, vs both (the round-3 kernel); OLS parity tests.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "ols or gaussian" > gpurun_out/r04h_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r04h_pytest.log
[ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
bash tools/gpu_bench_ab.sh r04h_a olsr3 4 2 || exit $?
bash tools/gpu_bench_ab.sh r04h_b ols2slot 4 1 || exit $?
bash tools/gpu_bench_ab.sh r04h_c ols2sync 4 1 || exit $?
DLSA_LIB=tools/_variants/libdlsa_hip_wnprof.so timeout -k 10 300 python -u tools/wn_prof.py > gpurun_out/r04h_wnprof.json 2> gpurun_out/r04h_wnprof.err || exit $?
cat gpurun_out/r04h_wnprof.json
