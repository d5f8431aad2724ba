# the driver's bench command on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/last
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err
