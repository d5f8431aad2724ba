# end-of-round measurements: full GPU parity suite, smoke, the default bench line and the other
# configs, rocprof kernel stats at C4 (Neal-8 and split-merge)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 880 --timeout-method thread -m gpu tests > $O/tests_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench_c5.jsonl 2> $O/bench_c5.err &&
timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline > $O/bench_c4.jsonl 2> $O/bench_c4.err &&
timeout -k 10 200 python -u bench.py --config c3 --no-cpu-baseline > $O/bench_c3.jsonl 2> $O/bench_c3.err &&
timeout -k 10 200 python -u bench.py --config c2 --no-cpu-baseline --steps 100 --warmup 10 > $O/bench_c2.jsonl 2> $O/bench_c2.err &&
timeout -k 10 200 python -u bench.py --init random20 --no-cpu-baseline --steps 10 --warmup 2 > $O/bench_c5r.jsonl 2> $O/bench_c5r.err &&
timeout -k 10 200 python -u bench.py --config c4 --sm --no-cpu-baseline --steps 30 --warmup 3 > $O/bench_c4_sm.jsonl 2> $O/bench_c4_sm.err &&
timeout -k 10 200 python -u bench.py --config c3 --sm --no-cpu-baseline --steps 60 --warmup 5 > $O/bench_c3_sm.jsonl 2> $O/bench_c3_sm.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline --steps 100 --warmup 5 > $O/prof_c4.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c4sm -o run --output-format csv -- python3 bench.py --config c4 --sm --no-cpu-baseline --steps 10 --warmup 3 > $O/prof_c4sm.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 > $O/prof_c5.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline --steps 100 --warmup 5 > $O/prof_c3.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c5r -o run --output-format csv -- python3 bench.py --init random20 --no-cpu-baseline --steps 10 --warmup 2 > $O/prof_c5r.log 2>&1
