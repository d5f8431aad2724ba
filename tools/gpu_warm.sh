# driver-window sensitivity: 20 timed steps after W warmup iterations
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/warm
mkdir -p $O
for w in 5 20 60 150; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup $w > $O/w$w.jsonl 2>/dev/null || exit 1
done
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 --warmup 5 > $O/s300w5.jsonl 2>/dev/null
