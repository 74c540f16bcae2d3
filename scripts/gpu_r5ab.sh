#!/bin/bash
# fp32 eval towers (key 19 = 0) with / without per-tap fragment addresses (AZG_EVAL_REMAT),
# then 2 vs 3 self-play groups.  scripts/_ab/libazg_pv_noremat.so was the product built with
# -DAZG_EVAL_REMAT=0 for this A/B only; it is not kept (rebuild it to rerun)
set -o pipefail
O=gpurun_out/r5ab; mkdir -p $O
A="--sp-games 0 --train-steps 0 --big-steps 0 --no-cpu-baseline --tune 19=0"
timeout -k 10 300 python -u bench.py $A > $O/remat1.log 2>&1 &&
AZG_PV_LIB=scripts/_ab/libazg_pv_noremat.so timeout -k 10 300 python -u bench.py $A > $O/remat0.log 2>&1 &&
timeout -k 10 300 python -u bench.py $A > $O/remat1b.log 2>&1 &&
AZG_PV_LIB=scripts/_ab/libazg_pv_noremat.so timeout -k 10 300 python -u bench.py $A > $O/remat0b.log 2>&1 &&
S="--skip-forward --no-cpu-baseline --train-steps 0 --big-steps 0"
AZG_SP_GROUPS=2 timeout -k 10 300 python -u bench.py $S > $O/g2.log 2>&1 &&
AZG_SP_GROUPS=3 timeout -k 10 300 python -u bench.py $S > $O/g3.log 2>&1 &&
AZG_SP_GROUPS=2 timeout -k 10 300 python -u bench.py $S > $O/g2b.log 2>&1 &&
AZG_SP_GROUPS=3 timeout -k 10 300 python -u bench.py $S > $O/g3b.log 2>&1
