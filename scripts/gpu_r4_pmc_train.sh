#!/bin/bash
# Round 4: PMC evidence for the train convs: separate rocprofv3
# --pmc passes over scripts/bench_train.py (6x128, B = 128, product schedule), plus a
# kernel trace of the same command (durations, scratch) and timing traces with the
# fused BN apply / finalize switched off (keys 23 / 24 = 0) to attribute their cost.
# -> python scripts/summarize_train_pmc_r4.py gpurun_out/pmc_train_r4 r4
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_train_r4
mkdir -p $OUT
CMD="python3 scripts/bench_train.py --steps 4 --warmup 2 --cpu-steps 0"
i=0
for pmc in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES" "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1
  s=$?; echo "pmc pass $i exit $s"; [ $s -eq 0 ] || exit $s
done
for t in default "23=0" "24=0"; do
  tune=""; [ "$t" != default ] && tune="--tune $t"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tr_${t/=/_} -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 $tune > $OUT/tr_${t/=/_}.log 2>&1
  s=$?; echo "trace $t exit $s"; [ $s -eq 0 ] || exit $s
done
echo done
