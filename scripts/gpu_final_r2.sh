#!/bin/bash
# Round-2 final evidence (profiles/):
#  sp     rocprofv3 kernel trace + stats of the headline self-play command
#  train  serial kernel trace (key 12 = 1) + PMC passes over the train step
#  conv   PMC passes of the per-layer conv at B=4096 (self-play's dominant kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/final_r2
mkdir -p $OUT/sp $OUT/train $OUT/conv
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/sp/trace -o run -- python3 bench.py --skip-forward --no-cpu-baseline --train-steps 0 --big-steps 0 > $OUT/sp/bench.json 2> $OUT/sp/bench.err
s=$?; echo "self-play trace exit $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/train/serial -o run -- python3 scripts/bench_train.py --steps 20 --cpu-steps 0 --serial > $OUT/train/serial.log 2>&1
s=$?; echo "train serial trace exit $s"; [ $s -eq 0 ] || exit $s
i=0
for pmc in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES" "SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/train/p$i -o run -- python3 scripts/bench_train.py --steps 4 --warmup 2 --cpu-steps 0 --serial > $OUT/train/p$i.log 2>&1
  s=$?; echo "train pmc $i exit $s"; [ $s -eq 0 ] || exit $s
done
for pmc in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/conv/pmc_$name -o run -- python3 scripts/conv_probe.py --batch 4096 --tower 0 --shape 8 --steps 2 > $OUT/conv/pmc_$name.log 2>&1
  s=$?; echo "conv pmc $pmc exit $s"; [ $s -eq 0 ] || exit $s
done
