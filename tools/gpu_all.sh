#!/bin/bash
# pytest -m gpu, then the config-2 bench + rocprof, then configs 5, 4 and 3.
# Usage: bash tools/gpu_all.sh <tag>
set -o pipefail
TAG=${1:-all}
bash tools/gpu_check.sh "$TAG" && CONFIGS="${CONFIGS:-5 4 3}" bash tools/bench_configs.sh "$TAG"
