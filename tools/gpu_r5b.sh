#!/bin/bash
# Round 5, run b: GPU suite + smoke on the options build, the DLSA_OZ_CHECK build's int8
# tests, per-wave exact-pass stamps (pass_bench base vs ozprof), the config-2 strong-scaling
# share (n = 1.25e7, K = 128) and its Newton-solve phase cycles (solveprof).
set -o pipefail
OUT=gpurun_out/${TAG:-r05b}; mkdir -p $OUT; export TMPDIR=/tmp
echo "[r5b] $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -1 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[r5b] $(date +%T) smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
echo "[r5b] $(date +%T) ozcheck int8 tests"
DLSA_LIB=var/libdlsa_hip_ozcheck.so timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -k "ozaki or config2" > $OUT/pytest_ozcheck.log 2>&1; rc=$?
tail -1 $OUT/pytest_ozcheck.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "[r5b] $(date +%T) pass_bench"
timeout -k 10 600 python -u tools/pass_bench.py --n 25000000 --p 100 --K 256 --rounds 3 --libs base,ozprof > $OUT/pass_bench.jsonl 2> $OUT/pass_bench.err || exit $?
cat $OUT/pass_bench.jsonl
echo "[r5b] $(date +%T) strong share"
timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --steps 10 --no-cpu-baseline > $OUT/bench_share8.json 2> $OUT/bench_share8.err || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['ms_per_step'],2), d.get('parity_rel'), d['stages_ms_per_step'], {k: round(v.get('ms_per_step', 0), 3) for k, v in d['kernels'].items()})" $OUT/bench_share8.json
echo "[r5b] $(date +%T) solveprof"
DLSA_LIB=var/libdlsa_hip_solveprof.so timeout -k 10 300 python -u bench.py --n 12500000 --partitions 128 --steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-fp64-step > $OUT/solveprof.json 2> $OUT/solveprof.err; rc=$?
grep -h "solve-profile" $OUT/solveprof.json $OUT/solveprof.err | head -12
[ $rc -eq 0 ] || exit $rc
echo "[r5b] $(date +%T) done"
