#!/bin/bash
# round 3, call D: fp32 MLP kernel A/B (LDS K-step balance, running bias corrections) + phase stamps
set -o pipefail
O=gpurun_out/r3x_d; mkdir -p $O
cd $GRAFT_REPO_ROOT
declare -A LIB=( [cur]=myfyp_amd/_native/libmyfyp_hip.so [base]=build/ab_P32_BALANCE0_P32_RUNNING_BC0/libmyfyp_hip.so [bc_only]=build/ab_P32_BALANCE0/libmyfyp_hip.so [bal_only]=build/ab_P32_RUNNING_BC0/libmyfyp_hip.so )
for pass in 1 2; do
  for v in cur base bc_only bal_only; do
    MYFYP_NATIVE_LIB=${LIB[$v]} timeout -k 10 120 python bench.py --steps 200 --warmup 10 > $O/bench_${v}_$pass.log 2>&1 || exit 1
  done
done
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so timeout -k 10 120 python scripts/probes/stamps_f32.py > $O/stamps_cur.log 2>&1 || exit 1
MYFYP_NATIVE_LIB=build/stamps_P32_BALANCE0_P32_RUNNING_BC0/libmyfyp_hip.so timeout -k 10 120 python scripts/probes/stamps_f32.py > $O/stamps_base.log 2>&1 || exit 1
