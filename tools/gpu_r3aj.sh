# round 3: short-list launches back on the one-wave resolver (C5/C3/C4 benches), tiny suite with
# the forced fixed-point resolver, and the A/B of the fixed-point workgroup (256 vs 512 threads)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3aj
mkdir -p $O
step() { "$@"; rc=$?; echo "rc $rc: $*" >> $O/steps.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_tiny.py > $O/tiny.log 2>&1
step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20.jsonl 2> $O/c5_20.err
step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300.jsonl 2> $O/c5_300.err
step timeout -k 10 120 python -u bench.py --config c3 --no-cpu-baseline > $O/c3.jsonl 2> $O/c3.err
step timeout -k 10 120 python -u bench.py --config c4 --no-cpu-baseline --steps 100 > $O/c4.jsonl 2> $O/c4.err
for v in base fp512; do
  if [ $v = base ]; then unset HDPM_LIB_VARIANT; else export HDPM_LIB_VARIANT=$v; fi
  step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2_$v.jsonl 2> $O/c2_$v.err
  step timeout -k 10 200 python -u bench.py --init random20 --no-cpu-baseline --steps 2 --warmup 1 > $O/c5r_$v.jsonl 2> $O/c5r_$v.err
done
exit 0
