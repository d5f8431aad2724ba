# round 3: pipelined sweeps + domain placement: full GPU suite, benches (C5 driver window x3,
# 300-step, C4, C3, C2), a kernel-trace profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; if [ $rc -ne 0 ] && [ -n "$STOP_ON_FAIL" ]; then exit $rc; fi; }
STOP_ON_FAIL=1 step timeout -k 10 90 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20a.jsonl 2> $O/c5_20a.err
step timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1
step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20b.jsonl 2> $O/c5_20b.err
step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20c.jsonl 2> $O/c5_20c.err
step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300.jsonl 2> $O/c5_300.err
HDPM_BENCH_TIMELINE=1 step timeout -k 10 120 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/c5_tl300.jsonl 2> $O/c5_tl300.err
step timeout -k 10 150 python -u bench.py --config c4 --steps 50 --warmup 5 --no-cpu-baseline > $O/c4.jsonl 2> $O/c4.err
step timeout -k 10 150 python -u bench.py --config c3 --steps 50 --warmup 5 --no-cpu-baseline > $O/c3.jsonl 2> $O/c3.err
step timeout -k 10 150 python -u bench.py --config c2 --no-cpu-baseline > $O/c2.jsonl 2> $O/c2.err
step timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/prof_c5.log 2>&1
exit 0
