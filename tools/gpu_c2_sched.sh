#!/bin/bash
# Config-2 Newton schedule probe: warm-start levels x approximate-Hessian precision,
# DLSA_TRACE per-iteration steps, bench ms and per-kernel times (no parity, no CPU leg).
set -o pipefail
OUT=gpurun_out/${TAG:-c2sched}; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # name hessian levels
  local name=$1 hs=$2 lv=$3
  DLSA_TRACE=1 DLSA_LEVELS="$lv" timeout -k 10 300 python -u bench.py --config 2 --steps 2 --warmup 1 \
      --no-cpu-baseline --no-parity --hessian $hs > $OUT/$name.json 2> $OUT/$name.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d['newton'], {k: (round(v.get('avg_launch_ms', 0), 3), v.get('launches_per_step')) for k, v in d['kernels'].items()})" $OUT/$name.json $name
  grep "dlsa trace" $OUT/$name.err | tail -12
}
run base mixed "${LV_BASE:-0.0625}"
run lv4 mixed 0.0625,0.25
run f32 mixed_f32 0.0625
run f32lv4 mixed_f32 0.0625,0.25
echo done
