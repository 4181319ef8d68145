#!/bin/bash
# r04e: GPU suite + config-2/5 bench on the current build, the exact-pass DMA
# schedule A/B, SQ counters of the config-4 OLS pass, config-3 traffic.
set -o pipefail
bash tools/gpu_suite.sh r04e 2 5 || exit $?
bash tools/gpu_oz_sched.sh r04e_sched || exit $?
bash tools/pmc.sh r04e_c4pmc --config 4 || exit $?
CONFIGS=3 bash tools/pmc_configs.sh r04e_pmc || exit $?
for LV in "0.25" "0.0625" "0.125,0.5" "0.5"; do
  DLSA_LEVELS=$LV timeout -k 10 300 python -u bench.py --config 5 --steps 3 --no-cpu-baseline \
      > gpurun_out/r04e/c5_lv_$LV.json 2> gpurun_out/r04e/c5_lv_$LV.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5 levels', sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], d['stages_ms_per_step'])" gpurun_out/r04e/c5_lv_$LV.json $LV
done
