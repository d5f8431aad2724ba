# round 3: unconverged regime profiles (C2, C5 random L=20) before the device-wide resolver
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; }
step timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --config c2 --no-cpu-baseline --steps 100 --warmup 20 > $O/prof_c2.log 2>&1
HDPM_BENCH_TIMELINE=1 step timeout -k 10 150 python -u bench.py --config c2 --no-cpu-baseline --steps 100 --warmup 20 > $O/c2_tl.jsonl 2> $O/c2_tl.err
step timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c5r -o run --output-format csv -- python3 bench.py --init random20 --no-cpu-baseline --steps 3 --warmup 1 > $O/prof_c5r.log 2>&1
exit 0
