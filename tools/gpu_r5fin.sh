#!/bin/bash
# Round 5: last check of the committed tree -- GPU suite, smoke, the default
# bench (config 2) and config 3.
set -o pipefail
OUT=gpurun_out/${TAG:-r05fin2}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit $?
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
timeout -k 10 400 python -u bench.py --config 3 --steps 4 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
for c in c2 c3; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],2), '%.3g' % d['value'], round(r['frac'],3), r.get('traffic'), d.get('parity_rel'))" $OUT/bench_$c.json $c; done
