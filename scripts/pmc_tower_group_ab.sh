cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pab
for g in 0 1; do
  for pmc in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $pmc -f csv -d gpurun_out/pab/g${g}_$pmc -o run -- python3 bench.py --steps 3 --warmup 1 --sp-games 0 --no-cpu-baseline --train-steps 0 --big-steps 0 --tune 5=1 --tune 6=8 --tune 17=$g > gpurun_out/pab/g${g}_$pmc.log 2>&1 || exit 1
  done
done
for g in 0 1; do timeout -k 10 100 python3 bench.py --steps 30 --warmup 5 --sp-games 0 --no-cpu-baseline --train-steps 0 --big-steps 0 --tune 5=1 --tune 6=8 --tune 17=$g 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('group', $g, d['forward_b512']['roofline']['frac'], d['forward_b512']['roofline']['avg_launch_us'])"; done
