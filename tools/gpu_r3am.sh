# round 3: first round from the snapshot draws (default): parity, A/B against bit 26 (stay)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3am
mkdir -p $O
step() { "$@"; rc=$?; echo "rc $rc: $*" >> $O/steps.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tiny.py > $O/tiny.log 2>&1
step timeout -k 10 400 python -u -m pytest -x -q --timeout 380 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "c2_full or random20" > $O/cfgpar.log 2>&1
step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2.jsonl 2> $O/c2.err
step timeout -k 10 200 python -u bench.py --init random20 --no-cpu-baseline --steps 3 --warmup 1 > $O/c5r.jsonl 2> $O/c5r.err
HDPM_BENCH_DEBUG=67108864 step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2_b26.jsonl 2> $O/c2_b26.err
HDPM_BENCH_DEBUG=67108864 step timeout -k 10 200 python -u bench.py --init random20 --no-cpu-baseline --steps 3 --warmup 1 > $O/c5r_b26.jsonl 2> $O/c5r_b26.err
HDPM_BENCH_DEBUG=2 step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline --steps 30 --warmup 10 > $O/c2_dbg.jsonl 2> $O/c2_dbg.err
exit 0
