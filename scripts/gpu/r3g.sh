#!/bin/bash
# round 3, call G: bisect the LL hand-offs (PL / dH2 separately) + the new CNN engine GPU tests
set -o pipefail
O=gpurun_out/r3x_g; mkdir -p $O
cd $GRAFT_REPO_ROOT
T="tests/test_mlp_f32_gpu.py::test_f32_epoch_matches_torch_adam"
for v in nn_P32_LL_PL0_P32_LL_DH20 pl_P32_LL_PL1_P32_LL_DH20 dh_P32_LL_PL0_P32_LL_DH21 main; do
  L=build/$v/libmyfyp_hip.so; [ $v = main ] && L=myfyp_amd/_native/libmyfyp_hip.so
  MYFYP_NATIVE_LIB=$L timeout -k 10 200 python -u -m pytest "$T" -q -x --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1; rc=$?; echo "$v rc=$rc" >> $O/status
  case $rc in 0|1) ;; *) exit $rc;; esac
done
timeout -k 10 400 python -u -m pytest tests/test_cnn_engine_gpu.py -v --timeout 200 --timeout-method thread > $O/cnn.log 2>&1; echo "cnn rc=$?" >> $O/status
