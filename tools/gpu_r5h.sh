#!/bin/bash
# Round 5, run h: presence pass with unconditional loads, cat pass with y in the row's
# single memory round trip: categorical GPU tests, config-3 benches and kernel trace.
set -o pipefail
OUT=gpurun_out/${TAG:-r05h}; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', v.get('ms_per_step', 0)), 3) for k, v in d['kernels'].items()}, {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" "$@"; }
echo "[r5h] $(date +%T) pytest"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "categorical or dummy or cat_ or ingest or airline" > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --config 3 --steps 4 --no-cpu-baseline > $OUT/bench_c3_$i.json 2> $OUT/bench_c3_$i.err || exit $?
  summ $OUT/bench_c3_$i.json c3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o run -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $OUT/prof_c3.json 2> $OUT/prof_c3.err || exit $?
python3 tools/kernel_sequence.py $OUT/prof_c3/run_results.db cat_ | head -10
echo "[r5h] $(date +%T) done"
