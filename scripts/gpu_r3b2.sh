#!/bin/bash
# Round 3: the default bench line on the final tree (roofline.traffic from the committed
# PMC records in profiles/conv_traffic.json, which must reach the box).
set -o pipefail
O=gpurun_out/r3b2
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
test -f profiles/conv_traffic.json || { echo "conv_traffic.json missing"; exit 1; }
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
s=$?; echo "bench rc $s"; tail -2 $O/bench.err; [ $s -eq 0 ] || exit $s
echo done
