#!/bin/bash
# round 4, call TPC: ResNet-18 weight-gradient split-K target (MYFYP_WGRAD_TPC) on the final tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4tpc; mkdir -p $O
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc $(grep -o '"value": [0-9.]*' $O/$n.log | tail -1)"; case $rc in 0) ;; *) exit $rc;; esac; }
R="python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1"
for k in a b c; do
  for t in 1 2 3; do MYFYP_WGRAD_TPC=$t run rn_tpc${t}_$k 300 $R; done
done
