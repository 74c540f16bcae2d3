#!/bin/bash
# Round 3 lease s: where the train forward conv's time goes -- kernel traces of the
# train step with the BN apply (key 23 = 0) or the BN finalize (key 24 = 0) outside
# the conv, against the defaults.
set -o pipefail
O=gpurun_out/r3s
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in default 23=0 24=0; do
  t=""; [ "$v" != default ] && t="--tune $v"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/tr_$v -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 $t > $O/tr_$v.log 2>&1
  s=$?; echo "trace $v rc $s"; [ $s -eq 0 ] || exit $s
done
echo done
