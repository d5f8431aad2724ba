# A/B of the wide prepass variants (HDPM_WIDE_VARIANT) at C4
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab_wide
mkdir -p $O
for r in 1 2; do
  for v in 0 1 2; do
    HDPM_WIDE_VARIANT=$v timeout -k 10 120 python bench.py --config c4 --no-cpu-baseline --steps 200 --warmup 10 > $O/b_${v}_$r.jsonl 2>/dev/null || exit 1
  done
done
HDPM_WIDE_VARIANT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k wide_prepass > $O/tests_v1.log 2>&1 &&
HDPM_WIDE_VARIANT=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k wide_prepass > $O/tests_v2.log 2>&1
