#!/bin/bash
# Round 4 lease b: per-item timeline of the persistent train backward (6x128, B = 128).
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python scripts/bwd_trace.py --run $O/trace.bin > $O/trace.txt 2>&1
s=$?; cat $O/trace.txt | head -60; [ $s -eq 0 ] || exit $s
echo done
