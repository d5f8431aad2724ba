# PMC passes (FETCH_SIZE, WRITE_SIZE: one counter per run) for the prepass at C5 and C4, the
# calibration kernel, and the kernel-trace stats of the default bench command
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc
mkdir -p $O
for c in c5 c4; do
  for k in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $k --kernel-trace -d $O/${c}_$k -o run --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --steps 5 --warmup 2 > $O/log_${c}_$k.txt 2>&1 || exit 1
  done
done
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/calib -o run --output-format csv -- ./tools/bin/fetch_calib > $O/log_calib.txt 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/stats_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/log_stats_c5.txt 2>&1
