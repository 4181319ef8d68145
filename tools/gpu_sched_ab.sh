#!/bin/bash
# Newton precision-schedule A/B on config 2 (DLSA_SCHED, warm-start levels):
# traced step sizes of one fit and the bench line for each setting.
# Usage: bash tools/gpu_sched_ab.sh <tag>
set -o pipefail
TAG=${1:-sched}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name env...
  local name=$1; shift
  env "$@" DLSA_TRACE=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline \
      > "$OUT/trace_$name.json" 2> "$OUT/trace_$name.err" || return $?
  grep "dlsa trace" "$OUT/trace_$name.err" | sed "s/^/$name /"
  env "$@" timeout -k 10 300 python -u bench.py --steps 4 --no-cpu-baseline > "$OUT/bench_$name.json" \
      2> "$OUT/bench_$name.err" || return $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" "$OUT/bench_$name.json" "$name"
}
run base DLSA_SCHED=0 &&
run sched DLSA_SCHED=1 &&
run sched_l4 DLSA_SCHED=1 DLSA_LEVELS=0.0625,0.25 DLSA_LEVEL_MAXIT=10,1 &&
run base_l4 DLSA_SCHED=0 DLSA_LEVELS=0.0625,0.25 DLSA_LEVEL_MAXIT=10,1
