mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in 0 4096; do
    HDPM_BENCH_DEBUG=$v timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --warmup 5 > gpurun_out/ab/b_${v}_$r.jsonl 2>/dev/null || exit 1
  done
done
