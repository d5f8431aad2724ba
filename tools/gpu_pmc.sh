# PMC passes (FETCH_SIZE, WRITE_SIZE: one counter per run, rocprofv3 does not split passes) of
# the prepass at C5 and C4, copied to gpurun_out/pmc/pmc_{fetch,write}_<config>.csv -- the files
# bench.py reads from profiles/<round>/ (PMC_ROUND) for roofline.traffic -- and the calibration
# kernel (tools/fetch_calib.hip: reported / true bytes of the access shapes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc
mkdir -p $O
for c in c5 c4; do
  for k in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $k --kernel-trace -d $O/${c}_$k -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 5 --warmup 2 > $O/log_${c}_$k.txt 2>&1 || exit 1
    f=$(find $O/${c}_$k -name "*counter_collection.csv" | head -1)
    [ -n "$f" ] && cp "$f" $O/pmc_$(echo $k | cut -d_ -f1 | tr 'A-Z' 'a-z')_$c.csv
  done
done
if [ -x tools/bin/fetch_calib ]; then
  timeout -k 10 60 ./tools/bin/fetch_calib > $O/fetch_calib.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/calib -o run --output-format csv -- ./tools/bin/fetch_calib > $O/log_calib.txt 2>&1 || exit 1
fi
