#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 300 python -u scripts/h3_bitwise_probe.py > $O/probe.log 2>&1
