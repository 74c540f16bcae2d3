#!/bin/bash
# SQ counters of the product towers (the lab's two passes, scripts/gpu_r5n.sh): MFMA busy,
# LDS-array busy, waits, LDS / VALU instructions per MFMA
# -> python scripts/summarize_h3_lab_pmc.py gpurun_out/r5s/<tag>
set -o pipefail
O=gpurun_out/r5s
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"
run() {   # tag, probe args
  tag=$1; shift; mkdir -p $O/$tag
  timeout -s KILL 120 rocprofv3 --pmc $P1 -f csv -d $O/$tag/p1 -o run -- python3 scripts/conv_probe.py "$@" --steps 2 > $O/$tag/p1.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc $P2 -f csv -d $O/$tag/p2 -o run -- python3 scripts/conv_probe.py "$@" --steps 2 > $O/$tag/p2.log 2>&1
}
run t_b3456 --batch 3456 --tower 1 --tower-shape 8 &&
run t12_b3456 --batch 3456 --tower 1 --tower-shape 12 &&
run t12_256_b512 --batch 512 --tower 1 --tower-shape 12 --blocks 10 --channels 256
