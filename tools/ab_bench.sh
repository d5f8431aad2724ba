# A/B of engine variants on the bench workload, interleaved: tools/ab_bench.sh OUTDIR "BITS_A BITS_B ..." [bench args]
# Each variant is an HDPM_BENCH_DEBUG value (include/hdpm.h hdpm_set_debug bits; 0 = default),
# three rounds, one JSON line per run under gpurun_out/OUTDIR.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
V=$2
shift 2
mkdir -p "$O"
for r in 1 2 3; do
  for v in $V; do
    HDPM_BENCH_DEBUG=$v timeout -k 10 150 python -u bench.py --no-cpu-baseline "$@" > "$O/b_${v}_$r.jsonl" 2> "$O/b_${v}_$r.err" || exit 1
  done
done
