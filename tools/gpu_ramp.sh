set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ramp
timeout -k 10 200 python -u tools/iter_times.py c5 5 60 > gpurun_out/ramp/iter_c5.json 2> gpurun_out/ramp/iter_c5.err &&
for r in 1 2 3; do timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/ramp/b20_$r.jsonl 2> gpurun_out/ramp/b20_$r.err || exit 1; done
