# round 3: the driver's 20-step window after the early torch context (x3), with timelines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; }
step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20a.jsonl 2> $O/c5_20a.err
step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20b.jsonl 2> $O/c5_20b.err
HDPM_BENCH_TIMELINE=1 step timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5_20tl.jsonl 2> $O/c5_20tl.err
HDPM_BENCH_TIMELINE=1 step timeout -k 10 120 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/c5_40tl.jsonl 2> $O/c5_40tl.err
step timeout -k 10 120 python -u bench.py --gpus 1 --no-cpu-baseline > $O/c5_default.jsonl 2> $O/c5_default.err
exit 0
