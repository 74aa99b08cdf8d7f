#!/bin/bash
# per-GPU layouts of the N = 2 / 4 / 8 mesh runs (4 / 2 / 1 peers of 7.5k samples each) on one GPU:
# K split 1 (single-XCD gangs, plain hand-offs) vs K split 2 (two-XCD gangs, write-through)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_ksab; mkdir -p $O
for k in a b; do
  for cfg in "4 30000" "2 15000" "1 7500"; do
    set -- $cfg
    for ks in 1 2; do
      MYFYP_F32_KS=$ks timeout -k 10 200 python bench.py --peers $1 --n-train $2 --steps 200 --warmup 10 > $O/p$1_ks${ks}_$k.log 2>&1; rc=$?
      echo "== peers $1 ks $ks ($k) rc=$rc $(grep -o '"value": [0-9.]*' $O/p$1_ks${ks}_$k.log)"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
