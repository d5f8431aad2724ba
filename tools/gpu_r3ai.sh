# round 3: A/B of the fixed-point resolver's workgroup (256 vs 512 threads: HDPM_LIB_VARIANT=fp512)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3ai
mkdir -p $O
step() { "$@"; rc=$?; echo "rc $rc: $*" >> $O/steps.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
for v in base fp512; do
  if [ $v = base ]; then unset HDPM_LIB_VARIANT; else export HDPM_LIB_VARIANT=$v; fi
  step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2_$v.jsonl 2> $O/c2_$v.err
  HDPM_BENCH_DEBUG=2 step timeout -k 10 200 python -u bench.py --init random20 --no-cpu-baseline --steps 2 --warmup 1 > $O/c5r_$v.jsonl 2> $O/c5r_$v.err
done
exit 0
