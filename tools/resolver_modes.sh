set -e
mkdir -p gpurun_out/r02q
for cfg in "c2 truth 30" "c2 random20 30" "c3 truth 30" "c5 random20 3" "c5 truth 100"; do
  set -- $cfg
  for dbg in 0 4096; do
    HDPM_BENCH_DEBUG=$dbg timeout -k 10 200 python bench.py --config $1 --init $2 --steps $3 --warmup 2 --no-cpu-baseline > gpurun_out/r02q/$1_$2_$dbg.jsonl 2> gpurun_out/r02q/$1_$2_$dbg.err
  done
done
