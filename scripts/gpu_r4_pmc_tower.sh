#!/bin/bash
# Round 4: where the 10x256 tower's HBM bytes go.  Study build,
# the 128x64 tower at B = 512 with halo_tile load ablations (key 8: 4 = no weight
# loads, 8 = no halo loads, 12 = neither) and with per-XCD-group claim queues (key
# 17 = 2), one counter group per pass:
# FETCH_SIZE (x2, gfx950) + WRITE_SIZE per launch.  6x128 at B = 3456 beside it.
set -o pipefail
export TMPDIR=/tmp AZG_PV_LIB=alphazero-gomoku_amd/libazg_pv_study.so
OUT=gpurun_out/pmc_r4
mkdir -p $OUT
run() {   # tag, probe args
  tag=$1; shift
  mkdir -p $OUT/$tag
  timeout -k 10 120 python3 scripts/conv_probe.py "$@" --steps 3 > $OUT/$tag/time.log 2>&1 || return 1
  for pmc in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/$tag/pmc_$pmc -o run -- python3 scripts/conv_probe.py "$@" --steps 2 > $OUT/$tag/pmc_$pmc.log 2>&1
    s=$?; echo "$tag pmc $pmc exit $s"; [ $s -eq 0 ] || return $s
  done
}
for abl in 0 4 8 12; do
  run t256_a$abl --batch 512 --tower 1 --tower-shape 8 --blocks 10 --channels 256 --abl $abl || exit 1
done
run t256_g2 --batch 512 --tower 1 --tower-shape 8 --blocks 10 --channels 256 --group 2 || exit 1
run t256_g0 --batch 512 --tower 1 --tower-shape 8 --blocks 10 --channels 256 --group 0 || exit 1
for abl in 0 4 8; do
  run t128_a$abl --batch 3456 --tower 1 --tower-shape 8 --abl $abl || exit 1
done
run t128_g2 --batch 3456 --tower 1 --tower-shape 8 --group 2 || exit 1
run t128_b512_g2 --batch 512 --tower 1 --tower-shape 8 --group 2 || exit 1
run t128_b512_g1 --batch 512 --tower 1 --tower-shape 8 --group 1 || exit 1
echo done
