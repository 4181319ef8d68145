#!/bin/bash
# Round 5, run ws: bench.py sizing the fit workspace before the warm-up -- bench tests, a config-2
# kernel trace (first full bf16 pass of every fit) and the config 2 / 3 / 5 lines.
set -o pipefail
OUT=gpurun_out/${TAG:-r05ws}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -k "bench" -q --timeout 300 --timeout-method thread > $OUT/pytest_bench.log 2>&1 || { tail -20 $OUT/pytest_bench.log; exit 1; }
tail -1 $OUT/pytest_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run -- python3 bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/prof_c2.json 2> $OUT/prof_c2.err || exit $?
python3 tools/kernel_sequence.py $OUT/prof_c2/run_results.db "irls_coop_kernel<7, 4, 0, false, 0, 1>"
for C in 2 3 5; do
  timeout -k 10 300 python -u bench.py --config $C --steps 4 --no-cpu-baseline > $OUT/bench_c$C.json 2> $OUT/bench_c$C.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" $OUT/bench_c$C.json c$C
done
