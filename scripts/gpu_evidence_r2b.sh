#!/bin/bash
# Round-2 (session 2) rocprofv3 evidence (profiles/r2b_*):
#  sp     kernel trace + stats of the headline bench command (self-play to game end)
#  train  overlapped kernel trace + stats, serial trace (key 12 = 1), PMC passes over it
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ev_r2b
mkdir -p $OUT/sp $OUT/train
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/sp/trace -o run -- python3 bench.py --skip-forward --no-cpu-baseline --train-steps 0 --big-steps 0 > $OUT/sp/bench.json 2> $OUT/sp/bench.err
s=$?; echo "self-play trace exit $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/train/trace -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $OUT/train/trace.log 2>&1
s=$?; echo "train trace exit $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/train/serial -o run -- python3 scripts/bench_train.py --steps 20 --cpu-steps 0 --serial > $OUT/train/serial.log 2>&1
s=$?; echo "train serial trace exit $s"; [ $s -eq 0 ] || exit $s
i=0
for pmc in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES" "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/train/pmc/p$i -o run -- python3 scripts/bench_train.py --steps 4 --warmup 2 --cpu-steps 0 --serial > $OUT/train/p$i.log 2>&1
  s=$?; echo "train pmc $i exit $s"; [ $s -eq 0 ] || exit $s
done
