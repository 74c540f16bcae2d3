#!/bin/bash
# Round 4 lease f: the 16-wave 128x128 tower tile at C = 256 (study build, key 6 = 10;
# key 10 = 1 the acquire form) against the 128x64 product tile: correctness, time and
# FETCH/WRITE traffic at 10x256, B = 512.
set -o pipefail
export TMPDIR=/tmp AZG_PV_LIB=alphazero-gomoku_amd/libazg_pv_study.so
OUT=gpurun_out/r4f
mkdir -p $OUT
timeout -k 10 120 python3 scripts/conv_probe.py --batch 64 --tower 1 --tower-shape 10 --blocks 10 --channels 256 --check --steps 1 > $OUT/check.log 2>&1; s=$?; tail -1 $OUT/check.log; [ $s -eq 0 ] || exit $s
run() {
  tag=$1; shift
  mkdir -p $OUT/$tag
  timeout -k 10 120 python3 scripts/conv_probe.py "$@" --steps 3 > $OUT/$tag/time.log 2>&1 || return 1
  tail -1 $OUT/$tag/time.log
  for pmc in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/$tag/pmc_$pmc -o run -- python3 scripts/conv_probe.py "$@" --steps 2 > $OUT/$tag/pmc_$pmc.log 2>&1
    s=$?; [ $s -eq 0 ] || return $s
  done
}
run s10 --batch 512 --tower 1 --tower-shape 10 --blocks 10 --channels 256 || exit 1
run s10a --batch 512 --tower 1 --tower-shape 10 --var 1 --blocks 10 --channels 256 || exit 1
run s8 --batch 512 --tower 1 --tower-shape 8 --blocks 10 --channels 256 || exit 1
echo done
