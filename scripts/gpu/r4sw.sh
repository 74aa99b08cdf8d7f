#!/bin/bash
# round 4, call SW: runtime-knob sweeps on the final tree — headline gather grid cap
# (MYFYP_PREP_GATHER_WGS) and the ResNet-18 BatchNorm accumulator row counts (MYFYP_BN_STAT_ROWS,
# MYFYP_BNB_ROWS); two runs per setting, alternated
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4sw; mkdir -p $O
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc $(grep -o '"value": [0-9.]*' $O/$n.log | tail -1)"; case $rc in 0) ;; *) exit $rc;; esac; }
for k in ${SW_KEYS:-a b}; do
  for w in ${SW_WGS:-32 64 128}; do MYFYP_PREP_GATHER_WGS=$w run mlp_w${w}_$k 200 python bench.py; done
done
R="python benchmarks/bench_cnn.py --model resnet18 --rounds 10 --warmup 1"
for k in ${SW_KEYS:-a b}; do
  for r in ${SW_ROWS:-8 16 32}; do MYFYP_BN_STAT_ROWS=$r MYFYP_BNB_ROWS=$r run rn_rows${r}_$k 300 $R; done
done
