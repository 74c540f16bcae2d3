#!/bin/bash
# configs[1] forward evidence (B = 512, persistent tower): kernel trace + PMC passes
# -> python scripts/summarize_profile.py $OUT/fwd <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/prof_fwd}
mkdir -p $OUT/fwd
FWD="bench.py --steps 20 --warmup 5 --sp-games 0 --no-cpu-baseline --train-steps 0 --big-steps 0"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/fwd/trace -o run -- python3 $FWD > $OUT/fwd/bench.json 2>&1
s=$?; echo "forward trace exit $s"; [ $s -eq 0 ] || exit $s
for pmc in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES"; do
  name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/fwd/pmc_$name -o run -- python3 bench.py --steps 3 --warmup 1 --sp-games 0 --no-cpu-baseline --train-steps 0 --big-steps 0 > $OUT/fwd/pmc_$name.log 2>&1
  s=$?; echo "pmc $pmc exit $s"; [ $s -eq 0 ] || exit $s
done
