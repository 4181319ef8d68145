#!/bin/bash
# Row-pass digit records (config 5): wide / int8 GPU tests with the digits from the row
# pass (default) and with the digits kernel (DLSA_WIDE_ROW_DIGITS=0), config-5 bench
# alternated, kernel trace.
set -o pipefail
OUT=gpurun_out/${TAG:-wdig}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "wide or config5 or ozaki" > $OUT/pytest_on.log 2>&1; rc=$?
tail -2 $OUT/pytest_on.log; grep -E "FAILED" $OUT/pytest_on.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  for arm in on off; do
    E="DLSA_AB_NONE=1"; [ $arm = off ] && E="DLSA_WIDE_ROW_DIGITS=0"
    env $E timeout -k 10 400 python -u bench.py --config 5 --steps 4 --no-cpu-baseline > $OUT/bench_c5_${arm}_$i.json 2> $OUT/bench_c5_${arm}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), d['newton'], {k: round(v.get('avg_launch_ms', v.get('ms_per_step',0)), 3) for k, v in d['kernels'].items()})" $OUT/bench_c5_${arm}_$i.json "c5 $arm"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $OUT/prof.json 2> $OUT/prof.err || exit $?
exit $rc
