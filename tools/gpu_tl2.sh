set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tl2
HDPM_BENCH_TIMELINE=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/tl2/s20.jsonl 2> gpurun_out/tl2/s20.err &&
HDPM_BENCH_TIMELINE=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 300 --warmup 5 > gpurun_out/tl2/s300.jsonl 2> gpurun_out/tl2/s300.err
