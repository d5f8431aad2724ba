set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/logt
timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_draws.py > gpurun_out/logt/t.log 2>&1
