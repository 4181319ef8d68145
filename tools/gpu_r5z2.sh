#!/bin/bash
# Round 5, run z2: bench.py releasing the previous step's outputs -- config 2 and 5 lines and a
# config-2 kernel trace (is the first full bf16 pass of every timed fit as fast as the others?).
set -o pipefail
OUT=gpurun_out/${TAG:-r05z2}; mkdir -p $OUT; export TMPDIR=/tmp
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()}, {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" "$@"; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
summ $OUT/bench_c2.json c2
timeout -k 10 300 python -u bench.py --config 5 --steps 4 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?
summ $OUT/bench_c5.json c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2 -o run -- python3 bench.py --config 2 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/prof_c2.json 2> $OUT/prof_c2.err || exit $?
python3 tools/kernel_sequence.py $OUT/prof_c2/run_results.db irls_ | awk '$4 > 1000000'
