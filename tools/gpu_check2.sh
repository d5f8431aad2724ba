set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-check2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 880 --timeout-method thread -m gpu tests > $O/tests_gpu.log 2>&1 &&
for r in 1 2 3; do
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b20_$r.jsonl 2>/dev/null || exit 1
  HDPM_BENCH_DEBUG=131072 timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/b20_off_$r.jsonl 2>/dev/null || exit 1
done &&
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/b300.jsonl 2>/dev/null
