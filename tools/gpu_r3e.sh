# round 3: early next-sweep preparation (speculative update_phi started before the commit and
# log-likelihood) and the lookahead copy of the next update's stream slice: parity + A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; }
step timeout -k 10 400 python -u -m pytest -v --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/parity.log 2>&1
step timeout -k 10 300 python -u -m pytest -v --maxfail=5 --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tiny.py > $O/tiny.log 2>&1
step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20a.jsonl 2> $O/c5_20a.err
step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20b.jsonl 2> $O/c5_20b.err
step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300.jsonl 2> $O/c5_300.err
HDPM_BENCH_DEBUG=2097152 step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300_oldorder.jsonl 2> $O/c5_300_oldorder.err
HDPM_BENCH_DEBUG=3145728 step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300_old.jsonl 2> $O/c5_300_old.err
HDPM_BENCH_DEBUG=2097152 step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20_oldorder.jsonl 2> $O/c5_20_oldorder.err
HDPM_BENCH_TIMELINE=1 step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_tl.jsonl 2> $O/c5_tl.err
HDPM_BENCH_TIMELINE=1 step timeout -k 10 120 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/c5_tl300.jsonl 2> $O/c5_tl300.err
exit 0
