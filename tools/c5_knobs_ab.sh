# C5 host-job and generator knobs (HDPM_HOST_THREADS, HDPM_MT_WORKGROUPS), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/c5knobs
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/c5_${tag}_$r.jsonl 2> $O/c5_${tag}_$r.err; }
for r in 1 2; do
  run def HDPM_X=0 || exit 1
  run mt128 HDPM_MT_WORKGROUPS=128 || exit 1
  run mt512 HDPM_MT_WORKGROUPS=512 || exit 1
  run ht12 HDPM_HOST_THREADS=12 || exit 1
  run ht6 HDPM_HOST_THREADS=6 || exit 1
done
