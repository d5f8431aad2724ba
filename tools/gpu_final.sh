# end-of-round GPU measurements, part 2: every config's bench line with both CPU baselines, the
# driver-style C5 window, and rocprof kernel stats (C5, C4, C3, C5 random-20, C4 + split-merge)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final6b
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_c5.jsonl 2> $O/bench_c5.err &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c5_driver.jsonl 2> $O/bench_c5_driver.err &&
timeout -k 10 300 python -u bench.py --config c4 > $O/bench_c4.jsonl 2> $O/bench_c4.err &&
timeout -k 10 300 python -u bench.py --config c3 > $O/bench_c3.jsonl 2> $O/bench_c3.err &&
timeout -k 10 300 python -u bench.py --config c2 --steps 100 --warmup 10 > $O/bench_c2.jsonl 2> $O/bench_c2.err &&
timeout -k 10 300 python -u bench.py --init random20 --steps 10 --warmup 2 > $O/bench_c5r.jsonl 2> $O/bench_c5r.err &&
timeout -k 10 300 python -u bench.py --config c4 --sm --steps 30 --warmup 3 > $O/bench_c4_sm.jsonl 2> $O/bench_c4_sm.err &&
timeout -k 10 300 python -u bench.py --config c3 --sm --steps 60 --warmup 5 > $O/bench_c3_sm.jsonl 2> $O/bench_c3_sm.err &&
timeout -k 10 200 python -u bench.py --config c4 --record --no-cpu-baseline > $O/bench_c4_record.jsonl 2> $O/bench_c4_record.err &&
timeout -k 10 200 python -u bench.py --record --no-cpu-baseline > $O/bench_c5_record.jsonl 2> $O/bench_c5_record.err &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 > $O/prof_c5.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python3 bench.py --config c4 --no-cpu-baseline --steps 100 --warmup 5 > $O/prof_c4.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --config c3 --no-cpu-baseline --steps 100 --warmup 5 > $O/prof_c3.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c5r -o run --output-format csv -- python3 bench.py --init random20 --no-cpu-baseline --steps 10 --warmup 2 > $O/prof_c5r.log 2>&1 &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c4sm -o run --output-format csv -- python3 bench.py --config c4 --sm --no-cpu-baseline --steps 10 --warmup 3 > $O/prof_c4sm.log 2>&1
