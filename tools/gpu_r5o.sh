#!/bin/bash
# Round 5, run o: OLS stream kernel with bounds-checked buffer loads: OLS tests, the
# FULL+STD debug comparison against the per-wave kernel, config-4 A/B, trace and PMC.
set -o pipefail
OUT=gpurun_out/${TAG:-r05o}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/ols_debug.py $OUT/ols_new.npz > $OUT/dbg_new.log 2>&1 || exit $?
DLSA_LIB=var/libdlsa_hip_olswave.so timeout -k 10 120 python -u tools/ols_debug.py $OUT/ols_old.npz > $OUT/dbg_old.log 2>&1 || exit $?
python3 -c "
import numpy as np
a=np.load('$OUT/ols_new.npz'); b=np.load('$OUT/ols_old.npz')
for k in a.files:
    d=np.abs(a[k]-b[k]).max()/max(np.abs(b[k]).max(),1e-300); print(k, d)
"
TAG=${TAG:-r05o} bash tools/gpu_r5n.sh
