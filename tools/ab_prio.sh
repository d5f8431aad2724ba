# A/B: stream priorities (sweep high, generator low) vs default priorities
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_prio
mkdir -p $O
for r in 1 2 3; do
  for v in 1 0; do
    HDPM_STREAM_PRIO=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/b20_${v}_$r.jsonl 2>/dev/null || exit 1
    HDPM_STREAM_PRIO=$v timeout -k 10 120 python bench.py --no-cpu-baseline > $O/b300_${v}_$r.jsonl 2>/dev/null || exit 1
  done
done
