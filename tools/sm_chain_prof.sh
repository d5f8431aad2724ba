# Split-merge device chain: host timeline and kernel stats at C4 and C3 (chain on / off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sm_prof
mkdir -p $O
for v in 1 0; do
  HDPM_SM_CHAIN=$v HDPM_BENCH_TIMELINE=1 timeout -k 10 200 python -u bench.py --config c4 --sm --no-cpu-baseline --steps 20 --warmup 3 > $O/tl_c4sm_$v.jsonl 2> $O/tl_c4sm_$v.err || exit 1
  HDPM_SM_CHAIN=$v HDPM_BENCH_TIMELINE=1 timeout -k 10 200 python -u bench.py --config c3 --sm --no-cpu-baseline --steps 40 --warmup 3 > $O/tl_c3sm_$v.jsonl 2> $O/tl_c3sm_$v.err || exit 1
done
HDPM_SM_CHAIN=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c4sm -o run --output-format csv -- python3 bench.py --config c4 --sm --no-cpu-baseline --steps 10 --warmup 3 > $O/prof_c4sm.log 2>&1 || exit 1
HDPM_SM_CHAIN=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c3sm -o run --output-format csv -- python3 bench.py --config c3 --sm --no-cpu-baseline --steps 20 --warmup 3 > $O/prof_c3sm.log 2>&1 || exit 1
