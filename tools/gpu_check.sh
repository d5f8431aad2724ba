set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 880 --timeout-method thread -m gpu tests > $O/tests_gpu.log 2>&1 &&
for r in 1 2; do timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_c5_$r.jsonl 2> $O/bench_c5_$r.err || exit 1; done &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/prof_c5.log 2>&1
