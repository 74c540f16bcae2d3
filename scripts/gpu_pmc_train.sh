#!/bin/bash
# PMC passes over the serial train step (weight grads on the caller's stream, key 12):
# per-kernel MFMA busy, LDS / wait profile and HBM fetch of conv3x3_train / wgrad
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_train2
mkdir -p $OUT
i=0
for pmc in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES" "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/p$i -o run -- python3 scripts/bench_train.py --steps 4 --warmup 2 --cpu-steps 0 --serial > $OUT/p$i.log 2>&1
  s=$?; echo "pmc pass $i exit $s"; [ $s -eq 0 ] || exit $s
done
