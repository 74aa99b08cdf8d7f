#!/bin/bash
# round 3, call H: LL hand-off dump probe (debug build) + the two retuned CNN numerics tests
set -o pipefail
O=gpurun_out/r3x_h; mkdir -p $O
cd $GRAFT_REPO_ROOT
MYFYP_NATIVE_LIB=build/dbg_P32_LL_DEBUG1_P32_LL_DH20/libmyfyp_hip.so timeout -k 10 200 python -u scripts/probes/ll_debug.py > $O/ll_debug.log 2>&1; echo "dbg rc=$?" >> $O/status
timeout -k 10 400 python -u -m pytest tests/test_cnn_engine_gpu.py -v --timeout 200 --timeout-method thread -k "lenet_train_step or trajectory" > $O/cnn.log 2>&1; echo "cnn rc=$?" >> $O/status
