#!/bin/bash
# Round-5 closing run: GPU suite, smoke, the default bench (config 2) and configs 3-5,
# the N=8 strong-scaling share of config 2, kernel traces (rocprofv3 --kernel-trace
# --stats) of configs 2-5, and HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE; one
# counter group per run) of configs 2, 3 and 4.
set -o pipefail
OUT=gpurun_out/${TAG:-r05z}; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['roofline'].get('frac'), {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)), 3) for k, v in d['kernels'].items()}, {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" "$@"; }
echo "[final] $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[final] $(date +%T) smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
echo "[final] $(date +%T) bench c2 (default)"
timeout -k 10 600 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
summ $OUT/bench_c2.json c2
for C in 3 4 5; do
  echo "[final] $(date +%T) bench c$C"
  timeout -k 10 400 python -u bench.py --config $C --steps 4 --no-cpu-baseline > $OUT/bench_c$C.json 2> $OUT/bench_c$C.err || exit $?
  summ $OUT/bench_c$C.json c$C
done
timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --steps 10 --no-cpu-baseline > $OUT/bench_c2_strong_share8.json 2> $OUT/bench_c2_strong_share8.err || exit $?
summ $OUT/bench_c2_strong_share8.json share8
for C in 2 3 4 5; do
  echo "[final] $(date +%T) kernel trace c$C"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c$C -o run -- python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/prof_c$C.json 2> $OUT/prof_c$C.err || exit $?
done
for C in 2 3 4; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    echo "[final] $(date +%T) pmc c$C $grp"
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_c$C/p$i -o run -- python3 bench.py --config $C --steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/pmc_c${C}_p$i.json 2> $OUT/pmc_c${C}_p$i.err || exit $?
  done
done
echo "[final] $(date +%T) done"
