#!/bin/bash
# int8 exact-pass GPU tests on variant builds (tools/_variants/libdlsa_hip_<v>.so), one
# pytest process per variant; stops on anything but a pass / test failure.
set -o pipefail
OUT=gpurun_out/${TAG:-varint8}; mkdir -p $OUT; export TMPDIR=/tmp
for v in $VARIANTS; do
  DLSA_LIB=tools/_variants/libdlsa_hip_$v.so timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "ozaki or config2" > $OUT/pytest_$v.log 2>&1; rc=$?
  echo "$v rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; grep FAILED $OUT/pytest_$v.log | head -5
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
