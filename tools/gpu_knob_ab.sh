#!/bin/bash
# bf16-pass knob A/B: pass timings and config-2 bench with and without $1 (ENV=VAL).
set -o pipefail
KN=$1
OUT=gpurun_out/${2:-knobab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "config1 or p100 or shapes or config2_shape" --timeout 240 --timeout-method thread > "$OUT/pytest_default.log" 2>&1 || { tail -3 "$OUT/pytest_default.log"; exit 1; }
env $KN timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "config1 or p100 or shapes or config2_shape" --timeout 240 --timeout-method thread > "$OUT/pytest_knob.log" 2>&1 || { tail -3 "$OUT/pytest_knob.log"; exit 1; }
tail -1 "$OUT/pytest_knob.log"
timeout -k 10 300 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --rounds 5 \
    --knobs "default;$KN" > "$OUT/ab_p100.jsonl" 2> "$OUT/ab_p100.err" && cat "$OUT/ab_p100.jsonl" || exit $?
for k in "" "$KN" "" "$KN"; do
  env $k timeout -k 10 300 python -u bench.py --config 2 --steps 5 --no-cpu-baseline --no-parity > "$OUT/c2.json" 2> "$OUT/c2.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" "$OUT/c2.json" "${k:-default}"
done
