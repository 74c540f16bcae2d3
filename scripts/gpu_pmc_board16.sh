#!/bin/bash
# PMC passes for the board16 roofline's `traffic` (MI355X_MICROARCH.md HBM section: one
# counter group per pass, FETCH_SIZE x2 + WRITE_SIZE) and its MFMA busy: the 16x16x32 board
# tower (key 19 = 2, the default at C = 128) at the self-play batch sizes 512 and 3,456.
# -> python scripts/summarize_board16_pmc.py gpurun_out/pmc_b16 r6 -> profiles/conv_traffic.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_b16
mkdir -p $OUT
run() {   # tag, probe args
  tag=$1; shift
  mkdir -p $OUT/$tag
  for pmc in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
    name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
    timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/$tag/pmc_$name -o run -- python3 scripts/conv_probe.py "$@" --steps 2 > $OUT/$tag/pmc_$name.log 2>&1
    s=$?; echo "$tag pmc $pmc exit $s"; [ $s -eq 0 ] || exit $s
  done
}
run b512 --batch 512 --tower 1 --tower-shape 14 || exit 1
run b3456 --batch 3456 --tower 1 --tower-shape 14 || exit 1
