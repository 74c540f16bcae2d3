#!/bin/bash
# Round 5: PMC + kernel-trace evidence for the weight-grad tile, v1 (key 48 = 0, round 4)
# vs v2 (key 48 = 1): the round-4 train PMC passes (scripts/gpu_r4_pmc_train.sh) over
# scripts/bench_train.py for both forms.
# -> python scripts/summarize_train_pmc_r4.py gpurun_out/r5_pmc_wgrad/v<k> r5_v<k>
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in 1 0; do
  OUT=gpurun_out/r5_pmc_wgrad/v$v
  mkdir -p $OUT
  CMD="python3 scripts/bench_train.py --steps 4 --warmup 2 --cpu-steps 0 --tune 48=$v"
  i=0
  for pmc in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES" "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
    s=$?; echo "v$v pmc pass $i exit $s"; [ $s -eq 0 ] || exit $s
  done
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tr_default -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 --tune 48=$v > $OUT/tr.log 2>&1
  s=$?; echo "v$v trace exit $s"; [ $s -eq 0 ] || exit $s
done
du -sh gpurun_out/r5_pmc_wgrad
echo done
