#!/bin/bash
# round 4, call Y: stride-2 dgrads as parity-class forward convs (MODE 5) with the compile-time
# epilogue operand sets + prefetch: CNN tests, ResNet-18 A/B MYFYP_CNN_S2_FWD=1 vs the default MODE 2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4y; mkdir -p $O
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -1 $O/$n.log | cut -c1-160; case $rc in 0) ;; *) exit $rc;; esac; }
run test_cnn 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_cnn_engine_gpu.py
R="python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1"
MYFYP_CNN_S2_FWD=1 run rn_new_a 300 $R
run rn_old_a 300 $R
MYFYP_CNN_S2_FWD=1 run rn_new_b 300 $R
run rn_old_b 300 $R
