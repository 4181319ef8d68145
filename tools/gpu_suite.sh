#!/bin/bash
# The whole GPU suite (all failures listed) then one config bench.
# Usage: bash tools/gpu_suite.sh <tag> [config ...]
set -o pipefail
TAG=${1:-suite}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[suite] $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for C in "$@"; do
  timeout -k 10 400 python -u bench.py --config $C --steps 4 --no-cpu-baseline > "$OUT/bench_c$C.json" 2> "$OUT/bench_c$C.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c'+sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v.get('avg_launch_ms', v.get('ms_per_step',0)), 3) for k, v in d['kernels'].items()})" "$OUT/bench_c$C.json" $C
done
exit $rc
