#!/bin/bash
# round 3, call F: bisect the fp32 MLP numerics failure (HEAD kernel = running BC only; LL without running BC; LL + BC)
set -o pipefail
O=gpurun_out/r3x_f; mkdir -p $O
cd $GRAFT_REPO_ROOT
T="tests/test_mlp_f32_gpu.py::test_f32_epoch_matches_torch_adam"
for v in headbc ll_P32_RUNNING_BC0 main; do
  L=build/$v/libmyfyp_hip.so; [ $v = main ] && L=myfyp_amd/_native/libmyfyp_hip.so
  MYFYP_NATIVE_LIB=$L timeout -k 10 200 python -u -m pytest "$T" -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1; echo "$v rc=$?" >> $O/status
done
