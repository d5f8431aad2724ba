# round 3: PMC pass on the fixed-point resolver at C5 random-20 (instruction mix and stalls)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3af
mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_IFETCH SQ_INSTS_LDS -d $O/pmc -o run --output-format csv -- python3 bench.py --init random20 --no-cpu-baseline --steps 1 --warmup 1 > $O/pmc.log 2>&1
echo "rc $?" >> $O/steps.log
exit 0
