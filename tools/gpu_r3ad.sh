# round 3: FP resolver phase timings incl. the draw share
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3ad
mkdir -p $O
step() { "$@"; rc=$?; echo "rc $rc: $*" >> $O/steps.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
HDPM_BENCH_DEBUG=2 step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline --steps 30 --warmup 10 > $O/c2_dbg.jsonl 2> $O/c2_dbg.err
HDPM_BENCH_DEBUG=2 step timeout -k 10 200 python -u bench.py --init random20 --no-cpu-baseline --steps 2 --warmup 1 > $O/c5r_dbg.jsonl 2> $O/c5r_dbg.err
exit 0
