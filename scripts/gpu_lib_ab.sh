#!/bin/bash
# Same-box A/B of two builds of the library (alphazero-gomoku_amd/libazg_pv_prev.so vs the
# current libazg_pv.so) on the board tower timings of scripts/board_abl.py, alternated
# twice (-> gpurun_out/lib_ab/ab.log)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lib_ab
mkdir -p $O
: > $O/ab.log
for r in 1 2; do
  for lib in prev cur; do
    if [ $lib = prev ]; then L=alphazero-gomoku_amd/libazg_pv_prev.so; else L=alphazero-gomoku_amd/libazg_pv.so; fi
    echo "== $lib round $r" >> $O/ab.log
    DUMP=$O/$lib AZG_PV_LIB=$L ABLS=0,0 timeout -k 10 200 python -u scripts/board_abl.py >> $O/ab.log 2>&1 || exit 1
  done
done
python -c "
import numpy as np
for B in (512, 3456):
    a, b = np.load('$O/prev_B%d.npy' % B), np.load('$O/cur_B%d.npy' % B)
    print('B=%d logits bitwise equal across builds:' % B, bool((a == b).all()), 'max diff', float(np.abs(a - b).max()))
" >> $O/ab.log
