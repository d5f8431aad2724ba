# round 3: pool workers spinning without registration: C5 windows + timeline, quick parity
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3t
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; }
step timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "update_phi or synthetic or iteration or zoo" > $O/parity.log 2>&1
step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20a.jsonl 2> $O/c5_20a.err
step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20b.jsonl 2> $O/c5_20b.err
HDPM_BENCH_TIMELINE=1 step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20tl.jsonl 2> $O/c5_20tl.err
step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300.jsonl 2> $O/c5_300.err
step timeout -k 10 120 python -u bench.py --config c4 --steps 50 --warmup 5 --no-cpu-baseline > $O/c4.jsonl 2> $O/c4.err
exit 0
