#!/bin/bash
# round 4, call ROWS: BN accumulator rows 16 -> 4 by default: CNN tests, ResNet-18 A/B against 16
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4rows; mkdir -p $O
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc $(grep -o '"value": [0-9.]*' $O/$n.log | tail -1)"; tail -1 $O/$n.log | cut -c1-100; case $rc in 0) ;; *) exit $rc;; esac; }
run test_cnn 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_cnn_engine_gpu.py tests/test_config5_gpu.py
R="python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1"
for k in a b; do
  run rn_new_$k 300 $R
  MYFYP_BN_STAT_ROWS=16 MYFYP_BNB_ROWS=16 run rn_old_$k 300 $R
done
