set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-sm1}
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "restricted or split_merge or logprobgs or hig" > $O/tests_sm.log 2>&1 &&
timeout -k 10 240 python -u bench.py --config c4 --sm --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c4_sm.jsonl 2> $O/bench_c4_sm.err &&
timeout -k 10 240 python -u bench.py --config c3 --sm --steps 60 --warmup 5 --no-cpu-baseline > $O/bench_c3_sm.jsonl 2> $O/bench_c3_sm.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c4sm --output-format csv -- python bench.py --config c4 --sm --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_c4sm.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 880 --timeout-method thread tests/test_gpu_configs.py -k "c4 or c3" > $O/tests_c34.log 2>&1 
