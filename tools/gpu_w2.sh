set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w3
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "wide or heads" > gpurun_out/w3/tests_wide.log 2>&1 &&
timeout -k 10 240 python -u bench.py --config c4 --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/w3/bench_c4.jsonl 2> gpurun_out/w3/bench_c4.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/w3/prof -o c4 --output-format csv -- python bench.py --config c4 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/w3/prof_c4.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 880 --timeout-method thread tests/test_gpu_configs.py -k c4 > gpurun_out/w3/tests_c4.log 2>&1
