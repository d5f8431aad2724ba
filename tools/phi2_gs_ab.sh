# group size of the fast device update (HDPM_PHI2_GS): C4, and C5 / C3 with the device update, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/phi2gs2
mkdir -p $O
for g in 32 64; do
  HDPM_PHI2_GS=$g timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_g${g}.jsonl 2> $O/c4_g${g}.err || exit 1
done
for g in 8 16 32; do
  HDPM_PHI2_GS=$g timeout -k 10 200 python -u bench.py --config c5 --phi device --no-cpu-baseline > $O/c5_g${g}.jsonl 2> $O/c5_g${g}.err || exit 1
  HDPM_PHI2_GS=$g timeout -k 10 200 python -u bench.py --config c3 --phi device --no-cpu-baseline > $O/c3_g${g}.jsonl 2> $O/c3_g${g}.err || exit 1
done
