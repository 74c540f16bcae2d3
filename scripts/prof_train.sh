cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/pt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/pt/serial -o run -- python3 scripts/bench_train.py --steps 10 --cpu-steps 0 --serial > gpurun_out/pt/serial.log 2>&1 && \
timeout -k 10 200 python3 scripts/bench_train.py --steps 20 --cpu-steps 0 > gpurun_out/pt/overlap.log 2>&1 && \
timeout -k 10 200 python3 scripts/bench_train.py --steps 20 --cpu-steps 0 --serial >> gpurun_out/pt/overlap.log 2>&1; cat gpurun_out/pt/overlap.log | grep -v amdgpu.ids
