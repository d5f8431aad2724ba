# locate the host fault in test_device_mt_stream_matches_r[1]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/segv
mkdir -p $O
python -c "import oracle_ffi" 2>/dev/null
HDPM_SEGV_TRACE=1 timeout -k 10 120 python -u tools/mt_repro.py 0 1 > $O/mt.log 2>&1
echo "rc $?" >> $O/mt.log
exit 0
