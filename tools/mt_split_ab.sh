# Stream windows generated in two launches (k_mt_jump + k_mt_twist, default) or one
# (k_mt_gen_multi, HDPM_MT_SPLIT=0): stream tests, then C5 / C4 bench lines, interleaved
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/mt_split
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  -k "mt_stream or c5_full or bench_path or keep_params" > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for v in 1 0; do
    HDPM_MT_SPLIT=$v timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/c5d_${v}_$r.jsonl 2> $O/c5d_${v}_$r.err || exit 1
  done
done
for v in 1 0; do
  HDPM_MT_SPLIT=$v timeout -k 10 120 python -u bench.py --no-cpu-baseline > $O/c5_${v}.jsonl 2> $O/c5_${v}.err || exit 1
  HDPM_MT_SPLIT=$v timeout -k 10 120 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_${v}.jsonl 2> $O/c4_${v}.err || exit 1
done
HDPM_MT_SPLIT=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 > $O/prof_c5.log 2>&1 || exit 1
