#!/bin/bash
# side-stream sizing beside the epoch: gather workgroups (MYFYP_PREP_GATHER_WGS) and evaluation cap (MYFYP_EVAL_WGS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_sideab; mkdir -p $O
for k in a b c; do
  for cfg in "64 32" "32 32" "16 32" "64 16"; do
    set -- $cfg
    MYFYP_PREP_GATHER_WGS=$1 MYFYP_EVAL_WGS=$2 timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/b_g$1_e$2_$k.log 2>&1; rc=$?
    echo "== gather $1 eval $2 ($k) rc=$rc $(grep -o '"value": [0-9.]*' $O/b_g$1_e$2_$k.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
