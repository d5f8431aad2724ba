# stream priorities (HDPM_STREAM_PRIO: 1 default = sweep and device update high, generator low;
# 2 = sweep at the generator's low priority, the device update high; 0 = all default) at C4, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/prio
mkdir -p $O
for r in 1 2; do
  for p in 1 2 0; do
    HDPM_STREAM_PRIO=$p timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_p${p}_$r.jsonl 2> $O/c4_p${p}_$r.err || exit 1
  done
done
