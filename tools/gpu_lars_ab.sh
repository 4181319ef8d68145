#!/bin/bash
# Host LARS A/B on the GPU box's CPU: tools/lars_time.py with the product
# library and tools/_variants/libdlsa_hip_larsold.so, alternated 3 times.
set -o pipefail
for r in 1 2 3; do
  for v in base larsold; do
    lib=$PWD/dlsa_amd/libdlsa_hip.so
    [ $v = base ] || lib=$PWD/tools/_variants/libdlsa_hip_$v.so
    echo "== $v"
    DLSA_LIB=$lib timeout -k 10 120 python -u tools/lars_time.py || exit $?
  done
done
