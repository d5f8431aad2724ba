# round 3: PMC passes on the device update_phi kernels (C5, device phi)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
HDPM_PHI=device timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU -d $O/pmc1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc1.log 2>&1 &&
HDPM_PHI=device timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/pmc2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc2.log 2>&1
