#!/bin/bash
# Round-2 rocprofv3 evidence:
#  prof_r2/sp     kernel trace + stats of the headline bench command (self-play to game end)
#  prof_r2/fwd    kernel trace of the configs[1] forward, then PMC passes on it
#                 (FETCH_SIZE, WRITE_SIZE, MFMA busy + clock, wave/LDS stats)
#  prof_r2/train  kernel trace of the train step (scripts/bench_train.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_r2
mkdir -p $OUT/sp $OUT/fwd $OUT/train
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/sp/trace -o run -- python3 bench.py --skip-forward --no-cpu-baseline --train-steps 0 --big-steps 0 > $OUT/sp/bench.json 2> $OUT/sp/bench.err
s=$?; echo "self-play trace exit $s"; tail -c 600 $OUT/sp/bench.json; [ $s -eq 0 ] || exit $s
FWD="bench.py --steps 20 --warmup 5 --sp-games 0 --no-cpu-baseline --train-steps 0 --big-steps 0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/fwd/trace -o run -- python3 $FWD > $OUT/fwd/bench.json 2>&1
s=$?; echo "forward trace exit $s"; [ $s -eq 0 ] || exit $s
for pmc in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
  name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/fwd/pmc_$name -o run -- python3 bench.py --steps 3 --warmup 1 --sp-games 0 --no-cpu-baseline --train-steps 0 --big-steps 0 > $OUT/fwd/pmc_$name.log 2>&1
  s=$?; echo "pmc $pmc exit $s"; [ $s -eq 0 ] || exit $s
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/train/trace -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > $OUT/train/trace.log 2>&1
s=$?; echo "train trace exit $s"; exit $s
