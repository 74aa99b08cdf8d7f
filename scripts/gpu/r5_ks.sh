#!/bin/bash
# fp32 epoch phase stamps at 8 / 2 / 1 peers per GPU (KS = 1 / 2 / 2): the per-GPU layouts of N = 1 / 4 / 8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5_ks; mkdir -p $O
for p in 8 2 1; do
  PEERS=$p MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so timeout -k 10 200 python scripts/probes/stamps_f32.py > $O/stamps_p$p.log 2>&1
  rc=$?; echo "== p$p rc=$rc"; grep -E "median|seen" $O/stamps_p$p.log; [ $rc -eq 0 ] || exit $rc
done
