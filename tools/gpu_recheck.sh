# re-check after the adapter's batch change: adapter replay and record tests, the driver's bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/recheck
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "adapter or record" > $O/tests.log 2>&1 &&
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.jsonl 2> $O/bench_driver.err &&
timeout -k 10 200 python -u bench.py --config c4 --record --no-cpu-baseline > $O/bench_c4_record.jsonl 2> $O/bench_c4_record.err
