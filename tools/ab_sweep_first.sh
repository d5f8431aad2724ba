# A/B: the prepared sweep launched before (32768) or after (0) the speculative update_phi
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_sf
for r in 1 2 3; do
  for v in 0 32768; do
    for c in c5 c4; do
      HDPM_BENCH_DEBUG=$v timeout -k 10 120 python bench.py --config $c --no-cpu-baseline --steps 300 --warmup 20 > gpurun_out/ab_sf/b_${c}_${v}_$r.jsonl 2>/dev/null || exit 1
    done
  done
done
