set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/cold
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/d20_$r.jsonl 2> $O/d20_$r.err || exit 1
done
timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/d300.jsonl 2> $O/d300.err || exit 1
timeout -k 10 120 python -u tools/iter_times.py c5 5 40 > $O/iter.json 2> $O/iter.err || exit 1
HDPM_BENCH_TIMELINE=1 timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/tl.jsonl 2> $O/tl.err || exit 1
