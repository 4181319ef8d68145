#!/bin/bash
# Ozaki-scheme exact pass bring-up: a first small parity test under a short
# limit, the exact-pass parity subset, then bench A/B against the fp64-MFMA
# exact pass (DLSA_OZ=0) at configs 2 and 4.
# Usage: bash tools/gpu_oz.sh <tag> [rounds]
set -o pipefail
TAG=${1:-oz}
R=${2:-1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[oz] $(date +%T) first test"
timeout -k 10 180 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -k "test_config1_vs_reference" > "$OUT/pytest_first.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_first.log"; [ $rc -eq 0 ] || exit $rc
echo "[oz] $(date +%T) parity subset"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    -k "config1 or p100 or shapes_vs_oracle or maxiter or ill_conditioned or stalled or config2_shape or edge_partitions or ols or standardized or games or exact_pass or misaligned or mixed_f32 or nonfinite or reference_signature or plain_c_abi" \
    > "$OUT/pytest_subset.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_subset.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for c in 2 4; do
  for i in $(seq 1 $R); do
    for arm in fp64 oz; do
      E="DLSA_AB_NONE=1"; [ $arm = fp64 ] && E="DLSA_OZ=0"
      env $E timeout -k 10 400 python -u bench.py --config $c --steps 4 --no-cpu-baseline \
          > "$OUT/bench_c${c}_${arm}_$i.json" 2> "$OUT/bench_c${c}_${arm}_$i.err" || exit $?
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v.get('ms_per_step', 0), 2) for k, v in d['kernels'].items()})" "$OUT/bench_c${c}_${arm}_$i.json" "c$c $arm"
    done
  done
done
echo "[oz] $(date +%T) done"
