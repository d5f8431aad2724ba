# round 3: C2 resolver-mode A/B, and the C2-C4 bench lines with their CPU baselines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O
step() { "$@"; rc=$?; if [ $rc -ge 124 ]; then echo "step rc $rc: $*" >> $O/steps.log; exit $rc; fi; echo "rc $rc: $*" >> $O/steps.log; }
step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2_default.jsonl 2> $O/c2_default.err
HDPM_BENCH_DEBUG=4096 step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2_noblk.jsonl 2> $O/c2_noblk.err
HDPM_BENCH_DEBUG=8192 step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline > $O/c2_blk.jsonl 2> $O/c2_blk.err
HDPM_BENCH_DEBUG=4128 step timeout -k 10 120 python -u bench.py --config c2 --no-cpu-baseline --steps 100 > $O/c2_noblk_tl.jsonl 2> $O/c2_noblk_tl.err
step timeout -k 10 240 python -u bench.py --config c2 > $O/c2_cpu.jsonl 2> $O/c2_cpu.err
step timeout -k 10 240 python -u bench.py --config c3 --steps 100 > $O/c3_cpu.jsonl 2> $O/c3_cpu.err
step timeout -k 10 300 python -u bench.py --config c4 --steps 100 > $O/c4_cpu.jsonl 2> $O/c4_cpu.err
exit 0
