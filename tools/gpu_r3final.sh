# round 3 final: full GPU suite, C5 driver-window + default bench, C2, C5 random-20, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3final
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; }
step timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/suite.log 2>&1
step timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/c5_20.jsonl 2> $O/c5_20.err
step timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300.jsonl 2> $O/c5_300.err
step timeout -k 10 120 python -u bench.py --config c2 > $O/c2.jsonl 2> $O/c2.err
step timeout -k 10 120 python -u bench.py --config c3 --no-cpu-baseline > $O/c3.jsonl 2> $O/c3.err
step timeout -k 10 120 python -u bench.py --config c4 --no-cpu-baseline --steps 100 > $O/c4.jsonl 2> $O/c4.err
step timeout -k 10 200 python -u bench.py --init random20 --no-cpu-baseline --steps 3 --warmup 1 > $O/c5r.jsonl 2> $O/c5r.err
step timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 10 > $O/prof.log 2>&1
step timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --config c2 --no-cpu-baseline --steps 100 --warmup 10 > $O/prof_c2.log 2>&1
exit 0
