#!/bin/bash
# r04g: GPU suite on the current build (OLS eta = 0, LARS slots), X-stream cache
# policy A/B at configs 2 and 4 (product nt vs dma0), HBM traffic of configs 2 and 4.
set -o pipefail
bash tools/gpu_suite.sh r04g 3 5; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_bench_ab.sh r04g_ab4 dma0 4 2 || exit $?
bash tools/gpu_bench_ab.sh r04g_ab2 dma0 2 2 || exit $?
OUT=gpurun_out/r04g_pmc
mkdir -p $OUT
for c in 2 4; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    for lib in base dma0; do
      L=""; [ $lib = dma0 ] && L=tools/_variants/libdlsa_hip_dma0.so
      echo "[pmc] $(date +%T) c$c $grp $lib"
      DLSA_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/c${c}_${grp}_$lib" -o run -- \
          python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-parity > "$OUT/c${c}_${grp}_$lib.json" 2> "$OUT/c${c}_${grp}_$lib.err" || exit $?
    done
  done
done
echo "[pmc] done"
