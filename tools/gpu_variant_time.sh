#!/bin/bash
# Exact-pass timing of variant builds against the product (tools/pass_bench.py, one process,
# interleaved rounds), then config-2 bench lines alternated product / BENCH_ALT.
set -o pipefail
OUT=gpurun_out/${TAG:-vartime}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --rounds ${ROUNDS:-3} \
    --libs $LIBS > $OUT/pass_bench.jsonl 2> $OUT/pass_bench.err || exit $?
cat $OUT/pass_bench.jsonl
for i in 1 2; do
  for v in base $BENCH_ALT; do
    if [ $v = base ]; then L=""; else L=tools/_variants/libdlsa_hip_$v.so; fi
    DLSA_LIB=$L timeout -k 10 300 python -u bench.py --config 2 --steps 3 --no-cpu-baseline --no-parity > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],2), {k: round(v.get('avg_launch_ms', 0), 3) for k, v in d['kernels'].items()})" $OUT/bench_${v}_$i.json $v
  done
done
