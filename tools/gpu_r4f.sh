#!/bin/bash
# r04f: the fixed heavy-tail test, exact-pass DMA schedule A/B, z-record A/B,
# config-4 SQ counters, config-3 traffic, config-5 level sweep.
set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 300 python -u -m pytest tests/test_gpu_ozaki.py -v --timeout 240 --timeout-method thread -k heavy \
    > gpurun_out/r04f/pytest_heavy.log 2>&1; tail -3 gpurun_out/r04f/pytest_heavy.log
bash tools/gpu_oz_sched.sh r04f_sched base,ozs1,ozs2,oz4d,oz4ds1,ozprof,ozs1prof,oz4dprof || exit $?
DLSA_LIB=tools/_variants/libdlsa_hip_oz4d.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ozaki.py tests/test_gpu_parity.py -v --timeout 240 --timeout-method thread -k "ozaki or exact_pass or config1 or p100" \
    > gpurun_out/r04f/pytest_oz4d.log 2>&1; tail -3 gpurun_out/r04f/pytest_oz4d.log
bash tools/gpu_env_ab.sh r04f_zrec DLSA_OZ_ZREC=0 2 2 || exit $?
bash tools/pmc.sh r04f_c4pmc --config 4 || exit $?
CONFIGS=3 bash tools/pmc_configs.sh r04f_pmc || exit $?
for LV in "0.25" "0.0625" "0.125,0.5" "0.5"; do
  DLSA_LEVELS=$LV timeout -k 10 300 python -u bench.py --config 5 --steps 3 --no-cpu-baseline \
      > gpurun_out/r04f/c5_lv_$LV.json 2> gpurun_out/r04f/c5_lv_$LV.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5 levels', sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], d['stages_ms_per_step'])" gpurun_out/r04f/c5_lv_$LV.json $LV
done
