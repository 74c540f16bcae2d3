#!/bin/bash
# Round-5 PMC passes (split-fp16 towers, key 19 = 1; same passes as rounds 3-4) for the rooflines' `traffic` (MI355X_MICROARCH.md HBM section:
# one counter group per pass, FETCH_SIZE x2 + WRITE_SIZE): the product tower at the
# self-play batch and at B = 512 (6x128), and the 10x256 tower at B = 512 (configs[4]);
# each pass is scripts/conv_probe.py with the tower forced to the shape the tuner picks.
# -> scripts/summarize_pmc_r3.py gpurun_out/pmc_r5 r5 -> profiles/conv_traffic.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_r5}
mkdir -p $OUT
run() {   # tag, probe args
  tag=$1; shift
  for pmc in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
    name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
    timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/$tag/pmc_$name -o run -- python3 scripts/conv_probe.py "$@" --steps 2 > $OUT/$tag/pmc_$name.log 2>&1
    s=$?; echo "$tag pmc $pmc exit $s"; [ $s -eq 0 ] || exit $s
  done
}
mkdir -p $OUT/t_b3456 $OUT/t_b512 $OUT/t_256_b512
run t_b3456 --batch 3456 --tower 1 --tower-shape ${SHAPE_128:-8} || exit 1
run t_b512 --batch 512 --tower 1 --tower-shape ${SHAPE_128:-8} || exit 1
run t_256_b512 --batch 512 --tower 1 --tower-shape ${SHAPE_256:-8} --blocks 10 --channels 256 || exit 1
