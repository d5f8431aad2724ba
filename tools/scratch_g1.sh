set -o pipefail
mkdir -p gpurun_out/r6a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "second_dataset or wide_scan_and_give_up or replica or tiny" > gpurun_out/r6a/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r6a/tests.log; exit 1; }
tail -3 gpurun_out/r6a/tests.log
for cfg in c5 c3 c4; do for phi in host device; do
  timeout -k 10 300 python -u bench.py --config $cfg --phi $phi --no-cpu-baseline > gpurun_out/r6a/bench_${cfg}_${phi}.jsonl 2> gpurun_out/r6a/bench_${cfg}_${phi}.err || { echo BENCHFAIL $cfg $phi; tail gpurun_out/r6a/bench_${cfg}_${phi}.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/r6a/bench_${cfg}_${phi}.jsonl')); print('$cfg $phi', d['value'], d['config']['fallbacks'], d['config']['update_phi'])"
done; done
