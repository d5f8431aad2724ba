# A/B of k_prepass_wide at C4 between the in-tree library and a variant build
# (HDPM_LIB_VARIANT=$1, split_and_merge_gibbs_sampling_amd/libhdpm_$1.so): kernel stats and two
# counter passes (SQ issue / wait cycles; L2 hits and misses) per build, under gpurun_out/ab_wide/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_wide
mkdir -p $O
V=$1
run() {   # tag, variant, rocprofv3 options...
  local tag=$1 var=$2
  shift 2
  HDPM_LIB_VARIANT=$var timeout -s KILL 120 rocprofv3 "$@" --kernel-trace -d $O/$tag -o run --output-format csv -- \
    python3 bench.py --config c4 --no-cpu-baseline --steps 30 --warmup 5 > $O/log_$tag.txt 2>&1
}
for var in "" "$V"; do
  t=${var:-new}
  run stats_$t "$var" --stats || exit 1
  run sq_$t "$var" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_IFETCH || exit 1
  run tcc_$t "$var" --pmc TCC_HIT_sum TCC_MISS_sum || exit 1
done
