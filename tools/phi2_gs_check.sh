# the fast update's group-size rule: device update parity tests, then C4 / C5-device / C3 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/phi2gs3
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
  -k "device_update_phi or bench_path or c3_full or c4_full or c5_full or split_merge_device_chain or restricted" > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_$r.jsonl 2> $O/c4_$r.err || exit 1
done
timeout -k 10 200 python -u bench.py --config c5 --phi device --no-cpu-baseline > $O/c5dev.jsonl 2> $O/c5dev.err || exit 1
timeout -k 10 200 python -u bench.py --config c5 --no-cpu-baseline > $O/c5.jsonl 2> $O/c5.err || exit 1
