#!/bin/bash
# Round-end check: smoke() and the whole GPU suite on the final build.
set -o pipefail
OUT=gpurun_out/${1:-final}
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[final] $(date +%T) smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
rc=$?; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
echo "[final] $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; grep -E "FAILED" "$OUT/pytest_gpu.log" | head
exit $rc
