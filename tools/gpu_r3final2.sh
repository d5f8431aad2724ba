# round 3 end: full GPU suite, smoke, C5 driver-window bench with CPU baseline, C2 bench, C5 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3final2
mkdir -p $O
step() { "$@"; rc=$?; echo "rc $rc: $*" >> $O/steps.log; if [ $rc -ge 124 ]; then exit $rc; fi; }
step timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
step timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/c5_20.jsonl 2> $O/c5_20.err
step timeout -k 10 120 python -u bench.py --config c2 > $O/c2.jsonl 2> $O/c2.err
step timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/prof.log 2>&1
exit 0
