#!/bin/bash
# Round 4 lease r: weight-grad side stream priority (key 51: 0 least = default, 1 greatest).
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
python -c "
import sys; sys.path[:0]=['.','alphazero-gomoku_amd']
import _native; lib=_native.load_library(); import torch; torch.zeros(1,device='cuda')
v=lib.azg_pv_set_tuning(51,-1); print('priority range least, greatest:', v//16 if v>=0 else -((-v)//16), (v%16)-8)"
for i in 1 2; do
  timeout -k 10 300 python -u scripts/train_r3_probe.py --ab "51=0;51=1" > $O/p$i.log 2>&1 || exit 1
  tail -1 $O/p$i.log | cut -c1-150
done
echo done
