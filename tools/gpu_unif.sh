set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/unif
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests_gpu.log 2>&1 &&
for v in 0 262144; do
  for c in c3 c5 c2 c4; do
    HDPM_BENCH_DEBUG=$v timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $O/b_${c}_$v.jsonl 2>/dev/null || exit 1
  done
  HDPM_BENCH_DEBUG=$v timeout -k 10 200 python -u bench.py --config c5 --init random20 --steps 3 --warmup 2 --no-cpu-baseline > $O/b_c5r20_$v.jsonl 2>/dev/null || exit 1
done
