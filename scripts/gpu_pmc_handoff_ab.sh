#!/bin/bash
# Where the round-2 tower traffic difference (2.08x with the acquire vs 1.75x with sc1
# loads, B = 512) came from: FETCH_SIZE / WRITE_SIZE of the 128x64 tower (study build)
# with (a) the acquire + 64-bit pointer loads (round-2 acquire form, VAR 0: 100 B/lane of
# scratch), (b) sc1 loads without the acquire (round-2 default, VAR 16: 32 B/lane), (c) the
# acquire + buffer addressing (product, VAR 32: no spill in the chunk loop), and the
# 16-wave tile with (d) sc1 loads (product) and (e) the acquire.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export AZG_PV_LIB=alphazero-gomoku_amd/libazg_pv_study.so
OUT=gpurun_out/pmc_handoff
mkdir -p $OUT
for cfg in "flat:8:13:0" "sc1:8:0:1" "buf:8:0:0" "w16sc1:10:0:0" "w16acq:10:1:0"; do
  IFS=: read tag shape var coh <<< "$cfg"
  mkdir -p $OUT/$tag
  for pmc in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d $OUT/$tag/pmc_$pmc -o run -- python3 scripts/conv_probe.py --batch 512 --tower 1 --tower-shape $shape --var $var --coh $coh --steps 2 > $OUT/$tag/pmc_$pmc.log 2>&1
    s=$?; echo "$tag pmc $pmc exit $s"; [ $s -eq 0 ] || exit $s
  done
done
