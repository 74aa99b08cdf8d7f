#!/bin/bash
# round 4, call C: phase stamps of the fp32 epoch, layout 1 vs layout 2, same box
set -o pipefail
O=gpurun_out/r4c; mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -3 $O/$n.log | cut -c1-400; case $rc in 0) ;; *) exit $rc;; esac; }
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so MYFYP_F32_VARIANT=2 run stamps_v2 200 python scripts/probes/stamps_f32v2.py
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so MYFYP_F32_VARIANT=1 run stamps_v1 200 python scripts/probes/stamps_f32.py
