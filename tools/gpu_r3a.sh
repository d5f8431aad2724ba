# round 3: small-N fixes (sweep_done), the bench-path parity test, the adapter replay
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tiny.py tests/test_gpu_adapter.py > $O/tiny.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 880 --timeout-method thread -m gpu tests/test_gpu_configs.py -k bench_path > $O/bench_path.log 2>&1
