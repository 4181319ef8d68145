#!/bin/bash
# Categorical pass ablations (tools/build_variants.sh cat*): config-3 bench per
# variant library, avg launch ms of cat_pass_kernel.  Usage: bash tools/gpu_cat_ab.sh <tag> <variants...>
set -o pipefail
TAG=${1:-catab}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in base "$@"; do
  lib=dlsa_amd/libdlsa_hip.so
  [ "$v" = base ] || lib=tools/_variants/libdlsa_hip_$v.so
  DLSA_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --config 3 --steps 3 --warmup 1 \
      --no-cpu-baseline --no-parity > "$OUT/bench_c3_$v.json" 2> "$OUT/bench_c3_$v.err" || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']['cat_pass_kernel']; print(sys.argv[2], round(d['ms_per_step'],2), {a: round(b,3) for a,b in k.items() if isinstance(b,float)})" "$OUT/bench_c3_$v.json" $v
done
