#!/bin/bash
# Same-box A/B of two library builds (libazg_pv_prev.so vs libazg_pv.so) on the bench's
# configs[1] forward and configs[2] self-play legs, alternated twice
# (-> gpurun_out/lib_bench_ab/*.json and summary.txt)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/lib_bench_ab
mkdir -p $O
: > $O/summary.txt
F="--no-cpu-baseline --sp32-games 0 --train-steps 0 --big-steps 0 --pente-moves 0"
for r in 1 2; do
  for lib in prev cur; do
    if [ $lib = prev ]; then L=alphazero-gomoku_amd/libazg_pv_prev.so; else L=alphazero-gomoku_amd/libazg_pv.so; fi
    AZG_PV_LIB=$L timeout -k 10 300 python3 -u bench.py $F > $O/${lib}_$r.json 2> $O/${lib}_$r.err || exit 1
    python3 -c "
import json; d=json.load(open('$O/${lib}_$r.json')); s=d['selfplay']['detail']; f=d['forward_b512']
print('$lib $r', 'selfplay', round(d['value']), 'busy', s['gpu_busy_share_rank0'], 'kernel ms', s['kernel_ms_rank0'],
      '| fwd512', f['boards_per_s'], f['ms_per_step'], f['kernel_ms_per_step'])" >> $O/summary.txt
  done
done
cat $O/summary.txt
