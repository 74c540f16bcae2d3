#!/bin/bash
# SQ counter passes (MFMA busy, LDS-array busy, waits, instruction mix) over one eval
# forward configuration: scripts/gpu_pmc_sq.sh <out-dir> <conv_probe.py args...>
# -> python scripts/summarize_h3_lab_pmc.py <out-dir>
set -o pipefail
O=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace -f csv -d $O/p1 -o run -- python3 scripts/conv_probe.py "$@" --steps 2 > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $P2 -f csv -d $O/p2 -o run -- python3 scripts/conv_probe.py "$@" --steps 2 > $O/p2.log 2>&1
