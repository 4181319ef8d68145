set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03l
timeout -k 10 300 python -u bench.py --config 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03l/b.json 2> gpurun_out/r03l/b.err
python3 -c "import json; d=json.load(open('gpurun_out/r03l/b.json')); print(d['newton'], d['ms_per_step'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03l/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity > /dev/null 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/r03l/prof -name "*kernel_stats.csv" | head -1 | xargs head -8 | cut -c1-150
