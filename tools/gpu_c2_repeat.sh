set -o pipefail
OUT=gpurun_out/r02g; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "config1 or p100 or categorical_vs or wide_shapes" --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --config 2 --steps 5 --no-cpu-baseline --no-parity > $OUT/c2_$i.json 2> $OUT/c2_$i.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['ms_per_step'],2), {k: round(v,2) for k,v in d['stages_ms_per_step'].items()}, {k: round(v.get('ms_per_step', 0), 2) for k, v in d['kernels'].items()})" $OUT/c2_$i.json
done
