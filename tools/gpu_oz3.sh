#!/bin/bash
# Ozaki exact pass (mixed mode): a first parity test under a short limit, the
# mixed-mode parity subset, then bench A/B against the fp64-MFMA exact pass.
# Usage: bash tools/gpu_oz3.sh <tag> [rounds]
set -o pipefail
TAG=${1:-oz3}
R=${2:-1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[oz3] $(date +%T) first test"
timeout -k 10 180 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -k "test_config1_vs_reference and mixed" > "$OUT/pytest_first.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_first.log"; [ $rc -eq 0 ] || exit $rc
echo "[oz3] $(date +%T) parity subset"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread \
    -k "config1 or p100 or shapes_vs_oracle or maxiter or ill_conditioned or stalled or config2_shape or edge_partitions or standardized or games or misaligned or nonfinite or reference_signature or plain_c_abi or scale or distributed" \
    > "$OUT/pytest_subset.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_subset.log"; grep -E "^E .*(assert|Error)|FAILED" "$OUT/pytest_subset.log" | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in $(seq 1 $R); do
  for arm in fp64 oz; do
    E="DLSA_AB_NONE=1"; [ $arm = fp64 ] && E="DLSA_OZ=0"
    env $E timeout -k 10 400 python -u bench.py --config 2 --steps 4 --no-cpu-baseline \
        > "$OUT/bench_c2_${arm}_$i.json" 2> "$OUT/bench_c2_${arm}_$i.err" || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v.get('ms_per_step', 0), 2) for k, v in d['kernels'].items()})" "$OUT/bench_c2_${arm}_$i.json" "c2 $arm"
  done
done
echo "[oz3] $(date +%T) done"
