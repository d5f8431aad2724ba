# launch shapes of the fast device update at C4 (environment knobs of launch_phi2), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/phi2knobs
mkdir -p $O
run() { # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_${tag}_$r.jsonl 2> $O/c4_${tag}_$r.err
}
for r in 1 2; do
  run def HDPM_X=0 || exit 1
  run g256 HDPM_PHI2_GROUP_THREADS=256 || exit 1
  run v8 HDPM_PHI2_VALUES_WAVES=8 || exit 1
  run t256 HDPM_PHI2_TREE_THREADS=256 || exit 1
  run g256v8 HDPM_PHI2_GROUP_THREADS=256 HDPM_PHI2_VALUES_WAVES=8 || exit 1
done
