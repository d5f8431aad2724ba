# A/B: update_phi phase B speculation batch (HDPM_PHI_SPEC 4 / 8 / 16 builds)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_spec2
mkdir -p $O
for r in 1 2; do
  for v in s4 s1 s2 s3; do
    if [ $v = s4 ]; then unset HDPM_LIB_VARIANT; else export HDPM_LIB_VARIANT=$v; fi
    for c in c5 c4; do
      HDPM_BENCH_TIMELINE=1 timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/b_${c}_${v}_$r.jsonl 2> $O/b_${c}_${v}_$r.err || exit 1
    done
  done
done
