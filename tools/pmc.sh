#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, each under its own time
# limit, as MI355X_MICROARCH.md prescribes) over a 1-step bench run.
# Usage: bash tools/pmc.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-pmc}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES"; do
  i=$((i+1))
  echo "[pmc] $(date +%T) pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > "$OUT/p$i.json" 2> "$OUT/p$i.err" || exit $?
done
echo "[pmc] done"
