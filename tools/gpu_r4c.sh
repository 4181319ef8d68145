#!/bin/bash
# r04c: GPU suite on the current build, then config-2 A/B against the round-4 start build.
set -o pipefail
bash tools/gpu_suite.sh r04c 5 || exit $?
bash tools/gpu_bench_ab.sh r04c r4base 2 2
