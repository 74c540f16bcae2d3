#!/bin/bash
# Round 6: self-play pipelining groups with the board16 forward -- the headline leg only,
# AZG_SP_GROUPS = 2 / 3 / 4 / 2 on one box (-> gpurun_out/r6n)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r6n
mkdir -p $O
for g in 2 3 4 2; do
  AZG_SP_GROUPS=$g timeout -k 10 300 python -u bench.py --skip-forward --no-cpu-baseline --train-steps 0 --big-steps 0 --sp32-games 0 > $O/g$g.json 2> $O/g$g.err || exit 1
  python -c "import json; d=json.loads(open('$O/g$g.json').read().strip().splitlines()[-1]); s=d['selfplay']['detail']; print('groups $g', d['value'], 'gpu busy', s['gpu_busy_share_rank0'], 'host wait', s['host_wait_share_rank0'])" >> $O/summary.txt
done
