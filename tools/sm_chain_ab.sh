# Split-merge device chain: its parity tests, then C4+SM / C3+SM with the chain on and off
# (HDPM_SM_CHAIN), interleaved, one JSON line per run under gpurun_out/sm_chain/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sm_chain
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  -k "split_merge or restricted or c3_full or c4_full" > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  for v in 1 0; do
    HDPM_SM_CHAIN=$v timeout -k 10 200 python -u bench.py --config c4 --sm --no-cpu-baseline --steps 30 --warmup 3 > $O/c4sm_${v}_$r.jsonl 2> $O/c4sm_${v}_$r.err || exit 1
    HDPM_SM_CHAIN=$v timeout -k 10 200 python -u bench.py --config c3 --sm --no-cpu-baseline --steps 60 --warmup 5 > $O/c3sm_${v}_$r.jsonl 2> $O/c3sm_${v}_$r.err || exit 1
  done
done
# stream windows started at the end of the current one (default) or at the current position
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export HDPM_WINDOW_FROM_NOW=1; else unset HDPM_WINDOW_FROM_NOW; fi
    timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5w_${v}_$r.jsonl 2> $O/c5w_${v}_$r.err || exit 1
  done
done
unset HDPM_WINDOW_FROM_NOW
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_300.jsonl 2> $O/c5_300.err || exit 1
timeout -k 10 120 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_300.jsonl 2> $O/c4_300.err || exit 1
