#!/bin/bash
# Round 5, run tr: the default bench (config 2) and config 3 after the PMC
# records were re-keyed to bench.py's kernel keys (roofline.traffic was null).
set -o pipefail
OUT=gpurun_out/${TAG:-r05tr}; mkdir -p $OUT
[ -n "$SKIP_C2" ] || timeout -k 10 600 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
timeout -k 10 400 python -u bench.py --config 3 --steps 4 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
for c in ${SUMM:-c2 c3}; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],2), r['frac'], r.get('traffic'), r.get('traffic_bytes_per_row'))" $OUT/bench_$c.json $c; done
