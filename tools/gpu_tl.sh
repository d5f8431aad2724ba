set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tl
HDPM_BENCH_TIMELINE=1 timeout -k 10 240 python -u bench.py --config c5 --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/tl/bench_c5.jsonl 2> gpurun_out/tl/bench_c5.err &&
HDPM_BENCH_TIMELINE=1 timeout -k 10 240 python -u bench.py --config c4 --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/tl/bench_c4.jsonl 2> gpurun_out/tl/bench_c4.err
