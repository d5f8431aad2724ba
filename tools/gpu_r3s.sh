# round 3: C2 resolver internal timings (debug bit 1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
HDPM_BENCH_DEBUG=2 timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline --steps 30 --warmup 10 > $O/c2_dbg.jsonl 2> $O/c2_dbg.err
echo "rc $?" >> $O/steps.log
exit 0
