#!/bin/bash
# Host WLSE + LARS timing at the config-5 size on the GPU box's host cores.
set -o pipefail
mkdir -p gpurun_out/lars
timeout -k 10 300 python -u tools/lars_bench.py > gpurun_out/lars/lars_bench.txt 2>&1; rc=$?
cat gpurun_out/lars/lars_bench.txt; exit $rc
