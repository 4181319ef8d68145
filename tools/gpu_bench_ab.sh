#!/bin/bash
# bench.py A/B of the product build against a variant, alternated.
# Usage: bash tools/gpu_bench_ab.sh <tag> <variant> <config> [rounds]
set -o pipefail
TAG=${1:-benchab}
V=$2
C=${3:-2}
R=${4:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in $(seq 1 $R); do
  for lib in base $V; do
    L=""; [ $lib = $V ] && L=tools/_variants/libdlsa_hip_$V.so
    DLSA_LIB=$L timeout -k 10 400 python -u bench.py --config $C --steps 4 --no-cpu-baseline \
        > "$OUT/bench_c${C}_${lib}_$i.json" 2> "$OUT/bench_c${C}_${lib}_$i.err" || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" "$OUT/bench_c${C}_${lib}_$i.json" "c$C $lib"
  done
done
