#!/bin/bash
# per-layer conv (self-play's dominant kernel) at B=4096: timing, then FETCH_SIZE /
# WRITE_SIZE passes for the roofline's traffic (profiles/conv_traffic.json)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_conv
mkdir -p $OUT
for b in 1024 2048 4096; do for t in 0 1; do
  timeout -k 10 120 python3 scripts/conv_probe.py --batch $b --tower $t --steps 10 2>&1 | grep -v amdgpu.ids || exit 1
done; done
for pmc in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
  name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/pmc_$name -o run -- python3 scripts/conv_probe.py --batch 4096 --tower 0 --steps 2 > $OUT/pmc_$name.log 2>&1
  s=$?; echo "pmc $pmc exit $s"; [ $s -eq 0 ] || exit $s
done
