set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 880 --timeout-method thread -m gpu tests > $O/tests_gpu.log 2>&1 &&
timeout -k 10 200 python -u tools/iter_times.py c5 5 20 > $O/iter_c5.json 2> $O/iter_c5.err &&
for r in 1 2 3; do timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > $O/b20_$r.jsonl 2> $O/b20_$r.err || exit 1; done &&
timeout -k 10 200 python -u bench.py > $O/b300.jsonl 2> $O/b300.err
