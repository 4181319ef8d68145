#!/bin/bash
# Round 5, run q: wide Newton kernel with one panel of lookahead and reciprocal pivots:
# the wide GPU tests, config-5 A/B against the round-4 panel sequence (wnold), kernel trace.
set -o pipefail
OUT=gpurun_out/${TAG:-r05q}; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()}, {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" "$@"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -k "wide or Wide" -x -v --timeout 240 --timeout-method thread > $OUT/pytest_wide.log 2>&1
rc=$?; tail -1 $OUT/pytest_wide.log; grep -E "FAILED|Error" $OUT/pytest_wide.log | head -20
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config 5 --steps 4 --no-cpu-baseline > $OUT/bench_c5_new_$r.json 2> $OUT/bench_c5_new_$r.err || exit $?
  summ $OUT/bench_c5_new_$r.json new$r
  DLSA_LIB=var/libdlsa_hip_wnold.so timeout -k 10 300 python -u bench.py --config 5 --steps 4 --no-cpu-baseline > $OUT/bench_c5_old_$r.json 2> $OUT/bench_c5_old_$r.err || exit $?
  summ $OUT/bench_c5_old_$r.json old$r
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o run -- python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/prof_c5.json 2> $OUT/prof_c5.err || exit $?
echo done
