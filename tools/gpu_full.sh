# full GPU parity suite (one process), then the launch-order A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 880 --timeout-method thread -m gpu tests > $O/tests_gpu.log 2>&1 &&
bash tools/ab_sweep_first.sh
