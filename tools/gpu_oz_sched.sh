#!/bin/bash
# Exact-pass DMA schedule A/B (tools/pass_bench.py, one process, interleaved rounds).
set -o pipefail
OUT=gpurun_out/${1:-ozsched}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --rounds 3 \
    --libs ${2:-base,ozs1,ozs2,ozprof,ozs1prof} > $OUT/pass_bench.jsonl 2> $OUT/pass_bench.err
rc=$?; cat $OUT/pass_bench.jsonl; tail -3 $OUT/pass_bench.err; exit $rc
