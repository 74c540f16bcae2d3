#!/bin/bash
# Kernel traces of the train step under tuning variants: TRACE_VARIANTS="24=0 23=0,24=0 ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tt
i=0
for v in ${TRACE_VARIANTS:-default}; do
  args=""
  if [ "$v" != "default" ]; then for kv in ${v//,/ }; do args="$args --tune $kv"; done; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tt/v$i -o run -- \
    python3 scripts/bench_train.py --steps 20 --cpu-steps 0 $args > gpurun_out/tt/v$i.log 2>&1
  s=$?; echo "trace $v exit $s"; [ $s -eq 0 ] || exit $s
  i=$((i+1))
done
