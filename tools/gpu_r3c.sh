# round 3: device update_phi (csrc/phi.hip) parity and first timings.  A step that times out
# or crashes (rc 124 / 134 / 137 / 139) ends the script; test failures (rc 1) do not.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; }
step timeout -k 10 500 python -u -m pytest -v --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "update_phi or zoo or synthetic" > $O/parity_phi.log 2>&1
step timeout -k 10 300 python -u -m pytest -v --maxfail=5 --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tiny.py > $O/tiny.log 2>&1
HDPM_PHI=device step timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_c5_dev.jsonl 2> $O/bench_c5_dev.err
HDPM_PHI=host step timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/bench_c5_host.jsonl 2> $O/bench_c5_host.err
HDPM_PHI=device step timeout -k 10 120 python -u bench.py --config c4 --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_c4_dev.jsonl 2> $O/bench_c4_dev.err
HDPM_PHI=host step timeout -k 10 120 python -u bench.py --config c4 --steps 50 --warmup 5 --no-cpu-baseline > $O/bench_c4_host.jsonl 2> $O/bench_c4_host.err
HDPM_PHI=device step timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > $O/prof_c5.log 2>&1
HDPM_PHI=device step timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline --steps 30 --warmup 5 > $O/prof_c4.log 2>&1
exit 0
