#!/bin/bash
# PMC passes over the serial train step (one counter group per run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_train
mkdir -p $OUT
i=0
for pmc in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU" \
           "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" ${EXTRA_PMC}; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -f csv -d $OUT/p$i -o run -- python3 scripts/bench_train.py --steps 3 --warmup 2 --cpu-steps 0 --serial ${TRAIN_ARGS} > $OUT/p$i.log 2>&1
  s=$?; echo "pmc pass $i exit $s"; [ $s -eq 0 ] || exit $s
done
