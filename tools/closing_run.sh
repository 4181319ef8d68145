#!/bin/bash
# The round's closing run through tools/gpu.sh: GPU suite, smoke, configs 2-5,
# the N = 8 per-rank share of config 2, kernel traces of configs 2-5 and the
# FETCH_SIZE / WRITE_SIZE passes (one counter per run) of configs 2-5.
#   TAG=r06z bash tools/closing_run.sh
# Summaries into profiles/: tools/rocpd_stats.py (kernel tables, written by the
# prof steps as <name>_kernel_stats.csv) and tools/pmc_summary.py (traffic ->
# profiles/pmc_traffic.json, which bench.py reads).
NOP="--no-cpu-baseline --no-parity --no-fp64-step"
steps=("test:" smoke "bench:bench_c2:")
for c in 3 4 5; do steps+=("bench:bench_c$c:--config $c --steps 4 --no-cpu-baseline"); done
steps+=("bench:bench_c2_strong_share8:--n 12500000 --partitions 128 --steps 10 --no-cpu-baseline")
for c in 2 3 4 5; do steps+=("prof:c$c:--config $c --steps 2 --warmup 1 $NOP"); done
for c in 2 3 4 5; do
  steps+=("pmc:c${c}_p1:FETCH_SIZE:--config $c --steps 1 --warmup 0 $NOP")
  steps+=("pmc:c${c}_p2:WRITE_SIZE:--config $c --steps 1 --warmup 0 $NOP")
done
exec bash "$(dirname "$0")/gpu.sh" "${steps[@]}"
