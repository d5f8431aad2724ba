# round 3: pipelined next sweep with the in-place scatter; timelines with medians.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; if [ $rc -ne 0 ] && [ -n "$STOP_ON_FAIL" ]; then exit $rc; fi; }
STOP_ON_FAIL=1 step timeout -k 10 90 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20a.jsonl 2> $O/c5_20a.err
step timeout -k 10 400 python -u -m pytest -v --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py -k "iterations or update_phi or synthetic" > $O/parity.log 2>&1
step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300.jsonl 2> $O/c5_300.err
HDPM_BENCH_DEBUG=4194304 step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300_nopipe.jsonl 2> $O/c5_300_nopipe.err
HDPM_BENCH_TIMELINE=1 step timeout -k 10 120 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/c5_tl300.jsonl 2> $O/c5_tl300.err
HDPM_BENCH_DEBUG=4194336 step timeout -k 10 120 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline > $O/c5_tl300_nopipe.jsonl 2> $O/c5_tl300_nopipe.err
step timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 > $O/prof_c5.log 2>&1
exit 0
