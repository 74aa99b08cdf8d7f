#!/bin/bash
# epoch graph vs direct launches of the epoch's kernels, after the single-XCD hand-offs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_direct; mkdir -p $O
for k in a b c d; do
  for v in 1 0; do
    MYFYP_EPOCH_GRAPH=$v timeout -k 10 200 python bench.py --steps 200 --warmup 10 > $O/b_graph${v}_$k.log 2>&1; rc=$?
    echo "== graph=$v ($k) rc=$rc $(grep -o '"value": [0-9.]*' $O/b_graph${v}_$k.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
for v in 1 0; do
  MYFYP_EPOCH_GRAPH=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b20_graph$v.log 2>&1; rc=$?
  echo "== 20 steps graph=$v rc=$rc $(grep -o '"value": [0-9.]*' $O/b20_graph$v.log)"; [ $rc -eq 0 ] || exit $rc
done
