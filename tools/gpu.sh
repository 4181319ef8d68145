#!/bin/bash
# One parameterised GPU runner for every measurement and A/B session (runs
# under gpurun; the library is built in-tree beforehand, never here).
#
#   TAG=r06x tools/gpu.sh STEP [STEP ...]
#
# Steps run in order; the first failure ends the run (no GPU step after a
# fault, abort or time limit).  Output goes to gpurun_out/$TAG/.
#
#   test:<pytest args>          GPU tests: pytest -m gpu <args> -> test_<n>.log (shell
#                               quoting inside the step: 'test:-k "config2 or config5"')
#   smoke                       __graft_entry__.smoke() -> smoke.log
#   bench:<name>:<bench args>   python bench.py <args> -> <name>.json + a summary line
#   prof:<name>:<bench args>    rocprofv3 --kernel-trace --stats of bench.py -> prof_<name>/
#                               and <name>_kernel_stats.csv (tools/rocpd_stats.py)
#   profpy:<name>:<script args> rocprofv3 --kernel-trace --stats of a Python script -> profpy_<name>/
#   trace:<name>:<bench args>   rocprofv3 --runtime-trace --kernel-trace (csv; no counters)
#                               -> trace_<name>/ (host API calls beside the kernels)
#   pmc:<name>:<counters>:<bench args>
#                               one rocprofv3 --pmc pass (counters comma-separated,
#                               within one block's limits) -> pmc_<name>/
#   py:<name>:<script args>     python -u <script args> -> <name>.txt (tools/*.py A/B helpers)
#   env:VAR=value               export for the following steps (e.g. DLSA_LIB=var/lib….so)
#   unenv:VAR                   unset it again
#
# Example (the round's closing run):
#   TAG=r06z tools/gpu.sh "test:" smoke "bench:c2:" "bench:c3:--config 3 --steps 4 --no-cpu-baseline" \
#       "prof:c2:--steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-fp64-step" \
#       "pmc:c2_fetch:FETCH_SIZE:--steps 1 --warmup 0 --no-cpu-baseline --no-parity --no-fp64-step"
set -o pipefail
OUT=gpurun_out/${TAG:?set TAG}; mkdir -p "$OUT"; export TMPDIR=/tmp
summ() {
  python3 - "$1" "$2" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
k = {n: round(v.get("avg_launch_ms", v.get("ms_per_step", 0)), 3) for n, v in d["kernels"].items()}
a = d.get("sig_inv_all_partitions", {})
print(sys.argv[2], round(d["ms_per_step"], 2), "%.4g" % d["value"], "frac", round(r["frac"], 3),
      "traffic", r.get("traffic"), "parity", d.get("parity_rel"), "allpart", a.get("max_elem_err"),
      k, {n: round(v, 3) for n, v in d.get("stages_ms_per_step", {}).items()})
EOF
}
ntest=0
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}
  echo "[gpu.sh] $(date +%T) $step"
  case $kind in
    test)
      ntest=$((ntest + 1))
      eval "targs=($rest)"  # shell quoting inside the step: test:-k "a or b"
      timeout -k 10 1200 python -u -m pytest tests -m gpu -v -rA --timeout 600 --timeout-method thread \
        "${targs[@]}" > "$OUT/test_$ntest.log" 2>&1
      rc=$?; tail -1 "$OUT/test_$ntest.log"; grep -E "^(FAILED|ERROR)" "$OUT/test_$ntest.log" | head -20
      [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > "$OUT/smoke.log" 2>&1 || exit $?
      tail -1 "$OUT/smoke.log" ;;
    bench)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 900 python -u bench.py $args > "$OUT/$name.json" 2> "$OUT/$name.err" || exit $?
      summ "$OUT/$name.json" "$name" ;;
    prof)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$name" -o run -- \
        python3 bench.py $args > "$OUT/prof_$name.json" 2> "$OUT/prof_$name.err" || exit $?
      db=$(find "$OUT/prof_$name" -name run_results.db | head -1)
      [ -n "$db" ] && python3 tools/rocpd_stats.py "$db" > "$OUT/${name}_kernel_stats.csv" && \
        head -8 "$OUT/${name}_kernel_stats.csv" ;;
    profpy)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/profpy_$name" -o run -- \
        python3 $args > "$OUT/profpy_$name.txt" 2> "$OUT/profpy_$name.err" || exit $?
      tail -12 "$OUT/profpy_$name.txt" ;;
    trace)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 600 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d "$OUT/trace_$name" \
        -o run -- python3 bench.py $args > "$OUT/trace_$name.json" 2> "$OUT/trace_$name.err" || exit $? ;;
    pmc)
      name=${rest%%:*}; rest=${rest#*:}; ctr=${rest%%:*}; args=${rest#*:}
      timeout -s KILL 180 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "$OUT/pmc_$name" -o run -- \
        python3 bench.py $args > "$OUT/pmc_$name.json" 2> "$OUT/pmc_$name.err" || exit $? ;;
    py)
      name=${rest%%:*}; args=${rest#*:}
      timeout -k 10 900 python -u $args > "$OUT/$name.txt" 2>&1 || exit $?
      tail -5 "$OUT/$name.txt" ;;
    env) export "$rest" ;;
    unenv) unset "$rest" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu.sh] $(date +%T) done"
