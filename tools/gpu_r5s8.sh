#!/bin/bash
# Round 5, run s8: kernel trace of the N=8 per-rank share of config 2 (where its 11 ms go) and the
# per-iteration Newton steps of config 5 (DLSA_TRACE).
set -o pipefail
OUT=gpurun_out/${TAG:-r05s8}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_s8 -o run -- python3 bench.py --n 12500000 --partitions 128 --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/prof_s8.json 2> $OUT/prof_s8.err || exit $?
DLSA_TRACE=1 timeout -k 10 200 python -u bench.py --config 5 --steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/c5_trace.json 2> $OUT/c5_trace.err || exit $?
grep "dlsa trace" $OUT/c5_trace.err | tail -12
