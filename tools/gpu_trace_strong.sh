#!/bin/bash
# Kernel trace (timestamps) of the config-2 strong-scaling per-rank share:
# where the per-fit fixed time goes.
set -o pipefail
OUT=gpurun_out/${1:-trace_strong}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/tr" -o run -- \
    python3 bench.py --scaling strong --n 12500000 --partitions 128 --steps 2 --warmup 1 --no-cpu-baseline --no-parity \
    > "$OUT/bench.json" 2> "$OUT/bench.err" && ls -R "$OUT/tr" | head
