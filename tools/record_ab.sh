# Recording every iteration (bench --record) in batches of 16 / 64 / 256 against the plain loop, same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/record6c
mkdir -p $O
for c in c5 c4; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline > $O/bench_$c.jsonl 2> $O/bench_$c.err || exit 1
  for b in 16 64 256; do
    HDPM_BENCH_RECORD_BATCH=$b timeout -k 10 200 python -u bench.py --config $c --record --no-cpu-baseline > $O/bench_${c}_record$b.jsonl 2> $O/bench_${c}_record$b.err || exit 1
  done
done
