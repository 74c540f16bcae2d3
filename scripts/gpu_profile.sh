#!/bin/bash
# rocprofv3 passes over the bench: kernel trace + stats, then separate PMC passes
# (HBM bytes: FETCH_SIZE and WRITE_SIZE each alone; MFMA busy + clock).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --sp-moves 0 --train-steps 0 --big-steps 0 ${BENCH_ARGS}"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/bench_trace.log 2>&1
s=$?; echo "trace exit $s"; tail -2 $OUT/bench_trace.log; [ $s -eq 0 ] || exit $s
for pmc in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" ${EXTRA_PMC}; do
  name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $pmc -f csv -d $OUT/pmc_$name -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --sp-moves 0 --train-steps 0 --big-steps 0 ${BENCH_ARGS} > $OUT/pmc_$name.log 2>&1
  s=$?; echo "pmc $pmc exit $s"; [ $s -eq 0 ] || exit $s
done
# train step (B=128) and the self-play leg (256 games x 400 sims): kernel traces only
mkdir -p gpurun_out/prof_${TAG}_train gpurun_out/prof_${TAG}_selfplay
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${TAG}_train/trace -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 > gpurun_out/prof_${TAG}_train/trace.log 2>&1
s=$?; echo "train trace exit $s"; [ $s -eq 0 ] || exit $s
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${TAG}_selfplay/trace -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --train-steps 0 --big-steps 0 > gpurun_out/prof_${TAG}_selfplay/trace.log 2>&1
s=$?; echo "selfplay trace exit $s"; [ $s -eq 0 ] || exit $s
# configs[4] network (10x256) forward: kernel trace only
mkdir -p gpurun_out/prof_${TAG}_big
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_${TAG}_big/trace -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --sp-moves 0 --train-steps 0 --big-steps 10 > gpurun_out/prof_${TAG}_big/trace.log 2>&1
s=$?; echo "big-net trace exit $s"; exit $s
