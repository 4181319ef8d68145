#!/bin/bash
# Round 5, run v: host LARS with the thread team (M = R^-1 products): timing at P = 100 / 182 / 500
# with the default team and one thread, then config 5 twice (stage wlse_lars_dbic).
set -o pipefail
OUT=gpurun_out/${TAG:-r05v}; mkdir -p $OUT; export TMPDIR=/tmp
nproc > $OUT/host.txt; python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> $OUT/host.txt
timeout -k 10 120 python -u tools/lars_time.py > $OUT/lars_team.txt 2>&1 || exit $?
DLSA_LARS_THREADS=1 timeout -k 10 120 python -u tools/lars_time.py > $OUT/lars_t1.txt 2>&1 || exit $?
cat $OUT/host.txt $OUT/lars_team.txt $OUT/lars_t1.txt
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config 5 --steps 4 --no-cpu-baseline > $OUT/bench_c5_$r.json 2> $OUT/bench_c5_$r.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['ms_per_step'],2), d.get('parity_rel'), {k: round(v, 3) for k, v in d.get('stages_ms_per_step', {}).items()})" $OUT/bench_c5_$r.json
done
