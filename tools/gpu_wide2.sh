set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/wide2
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "wide or heads" > $O/tests_wide.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 880 --timeout-method thread tests/test_gpu_configs.py -k c4 > $O/tests_c4.log 2>&1 &&
for r in 1 2; do timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline > $O/bench_c4_$r.jsonl 2>/dev/null || exit 1; done &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c4 --output-format csv -- python3 bench.py --config c4 --steps 100 --warmup 5 --no-cpu-baseline > $O/prof_c4.log 2>&1
