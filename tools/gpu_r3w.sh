# round 3: fixed-point resolver (k_resolve_fp): parity (tiny, parity, C2 modes, C5 random-20), C2 / C5-random / C5 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O
step() { "$@"; rc=$?; echo "rc $rc: $*" >> $O/steps.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tiny.py > $O/tiny.log 2>&1
step timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "c2_full" > $O/c2par.log 2>&1
step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2.jsonl 2> $O/c2.err
step timeout -k 10 200 python -u bench.py --init random20 --no-cpu-baseline --steps 3 --warmup 1 > $O/c5r.jsonl 2> $O/c5r.err
step timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/parity.log 2>&1
step timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "random20" > $O/c5rpar.log 2>&1
exit 0
