# round 3: resolver LIST mode with staged rows: parity (resolver-heavy tests) + C2 / C5-random timings
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3p
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; }
step timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_tiny.py > $O/parity.log 2>&1
step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2.jsonl 2> $O/c2.err
HDPM_BENCH_DEBUG=32 step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline --steps 100 > $O/c2_tl.jsonl 2> $O/c2_tl.err
step timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --config c2 --no-cpu-baseline --steps 100 --warmup 20 > $O/prof_c2.log 2>&1
step timeout -k 10 200 python -u bench.py --init random20 --no-cpu-baseline --steps 3 --warmup 1 > $O/c5r.jsonl 2> $O/c5r.err
exit 0
