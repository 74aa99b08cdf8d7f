#!/bin/bash
# round 4, call FF: fused BN finalize (MYFYP_CNN_FUSE_FIN=1) re-measured with the 4-row accumulators
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4ff; mkdir -p $O
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc $(grep -o '"value": [0-9.]*' $O/$n.log | tail -1)"; case $rc in 0) ;; *) exit $rc;; esac; }
R="python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1"
for k in a b c; do
  MYFYP_CNN_FUSE_FIN=1 run rn_fused_$k 300 $R
  run rn_sep_$k 300 $R
done
