# round 3: full GPU suite after the small-N fix; driver-window bench lines; kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/tests_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_c5_drv.jsonl 2> $O/bench_c5_drv.err &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c5_drv2.jsonl 2>> $O/bench_c5_drv.err &&
timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/bench_c5_300.jsonl 2>> $O/bench_c5_drv.err &&
HDPM_BENCH_TIMELINE=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c5_tl.jsonl 2> $O/bench_c5_tl.err &&
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/trace_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/trace_c5.log 2>&1
