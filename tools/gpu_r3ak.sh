# round 3: the fixed-point resolver at 512 threads (default): parity; A/B against 1024 threads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3ak
mkdir -p $O
step() { "$@"; rc=$?; echo "rc $rc: $*" >> $O/steps.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tiny.py > $O/tiny.log 2>&1
step timeout -k 10 400 python -u -m pytest -x -q --timeout 380 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "c2_full or random20" > $O/cfgpar.log 2>&1
for v in base fp1024; do
  if [ $v = base ]; then unset HDPM_LIB_VARIANT; else export HDPM_LIB_VARIANT=$v; fi
  step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2_$v.jsonl 2> $O/c2_$v.err
  step timeout -k 10 200 python -u bench.py --init random20 --no-cpu-baseline --steps 3 --warmup 1 > $O/c5r_$v.jsonl 2> $O/c5r_$v.err
done
unset HDPM_LIB_VARIANT
HDPM_BENCH_DEBUG=2 step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline --steps 30 --warmup 10 > $O/c2_dbg.jsonl 2> $O/c2_dbg.err
exit 0
