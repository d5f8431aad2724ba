# A/B of k_prepass_wide at C4 between environment settings of the in-tree library:
# bash tools/ab_wide_env.sh "VAR=a" "VAR=b" ... -> kernel traces under gpurun_out/ab_env/<i>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_env
mkdir -p $O
i=0
for kv in "$@"; do
  i=$((i + 1))
  env $kv true || exit 1
  export $kv
  timeout -s KILL 120 rocprofv3 --stats --kernel-trace -d $O/$i -o run --output-format csv -- \
    python3 bench.py --config c4 --no-cpu-baseline --steps 60 --warmup 5 > $O/log_$i.txt 2>&1 || exit 1
  echo "$kv" > $O/$i/setting.txt
done
