set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tlsm
HDPM_BENCH_TIMELINE=1 timeout -k 10 200 python -u bench.py --config c4 --sm --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/tlsm/c4.jsonl 2> gpurun_out/tlsm/c4.err
