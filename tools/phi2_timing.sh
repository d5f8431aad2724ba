# phase marks of the fast device update at C4 (synchronous updates: HDPM_BENCH_DEBUG=128)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/phi2t
mkdir -p $O
HDPM_PHI_TIMING=1 HDPM_BENCH_DEBUG=128 timeout -k 10 200 python -u bench.py --config c4 --phi device --steps 30 --warmup 3 --no-cpu-baseline > $O/c4.jsonl 2> $O/c4.err || exit 1
HDPM_PHI_TIMING=1 HDPM_BENCH_DEBUG=128 timeout -k 10 200 python -u bench.py --config c5 --phi device --steps 30 --warmup 3 --no-cpu-baseline > $O/c5.jsonl 2> $O/c5.err || exit 1
