#!/bin/bash
# pytest -m gpu, then the config-2 bench + rocprof, then configs 5 and 4.
# Usage: bash tools/gpu_all.sh <tag>
set -o pipefail
TAG=${1:-all}
bash tools/gpu_check.sh "$TAG" && CONFIGS="5 4" bash tools/bench_configs.sh "$TAG"
