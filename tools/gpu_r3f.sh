# round 3: the next sweep enqueued ahead (pre_enqueue / k_pipe_wait / pipe_go): a short bench
# first (bounded), then parity, then A/B benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; if [ $rc -ne 0 ] && [ -n "$STOP_ON_FAIL" ]; then exit $rc; fi; }
STOP_ON_FAIL=1 step timeout -k 10 90 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20a.jsonl 2> $O/c5_20a.err
step timeout -k 10 400 python -u -m pytest -v --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/parity.log 2>&1
step timeout -k 10 300 python -u -m pytest -v --maxfail=5 --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tiny.py > $O/tiny.log 2>&1
step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20b.jsonl 2> $O/c5_20b.err
step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300.jsonl 2> $O/c5_300.err
HDPM_BENCH_DEBUG=4194304 step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300_nopipe.jsonl 2> $O/c5_300_nopipe.err
HDPM_BENCH_DEBUG=4194304 step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20_nopipe.jsonl 2> $O/c5_20_nopipe.err
HDPM_BENCH_TIMELINE=1 step timeout -k 10 120 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/c5_tl300.jsonl 2> $O/c5_tl300.err
step timeout -k 10 120 python -u bench.py --config c4 --steps 50 --warmup 5 --no-cpu-baseline > $O/c4.jsonl 2> $O/c4.err
step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2.jsonl 2> $O/c2.err
exit 0
