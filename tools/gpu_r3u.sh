# round 3: prepass streaming loads non-temporal (pool heads kept in cache) A/B: kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; }
for v in base nt base nt; do
HDPM_LIB_VARIANT=$v step timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run_$RANDOM --output-format csv -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/b_$v.log 2>&1
done
exit 0
