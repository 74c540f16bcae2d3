#!/bin/bash
# per-layer conv (self-play's dominant kernel, forced 128x64 / 8 waves) at B=4096:
# FETCH_SIZE / WRITE_SIZE / MFMA-busy passes for the roofline's traffic
# (scripts/summarize_conv_pmc.py -> profiles/conv_traffic.json)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_conv8
mkdir -p $OUT
for pmc in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/pmc_$name -o run -- python3 scripts/conv_probe.py --batch 4096 --tower 0 --shape 8 --steps 2 > $OUT/pmc_$name.log 2>&1
  s=$?; echo "pmc $pmc exit $s"; [ $s -eq 0 ] || exit $s
done
