#!/bin/bash
# Round 5, run n: OLS pass streaming X into the MFMA operand registers (ols_stream.hip,
# product) vs the per-wave LDS-DMA kernel (olswave): OLS GPU tests, config-4 benches,
# kernel trace and PMC traffic of the new kernel.
set -o pipefail
OUT=gpurun_out/${TAG:-r05n}; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['roofline'].get('frac'), {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)), 3) for k, v in d['kernels'].items()}, {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" "$@"; }
echo "[r5n] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "ols or OLS or gaussian or config4 or linear" > $OUT/pytest_ols.log 2>&1
rc=$?; tail -1 $OUT/pytest_ols.log; grep -E "FAILED" $OUT/pytest_ols.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for v in base olswave; do
    if [ $v = base ]; then L=""; else L=var/libdlsa_hip_$v.so; fi
    DLSA_LIB=$L timeout -k 10 300 python -u bench.py --config 4 --steps 5 --no-cpu-baseline > $OUT/bench_c4_${v}_$i.json 2> $OUT/bench_c4_${v}_$i.err || exit $?
    summ $OUT/bench_c4_${v}_$i.json c4_$v
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o run -- python3 bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $OUT/prof_c4.json 2> $OUT/prof_c4.err || exit $?
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_c4/p$i -o run -- python3 bench.py --config 4 --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $OUT/pmc_c4_p$i.json 2> $OUT/pmc_c4_p$i.err || exit $?
done
echo "[r5n] $(date +%T) done"
