#!/bin/bash
# round 4, call F: layout-2 stamps after spreading the W3 / b3 updates; bench A/B
set -o pipefail
O=gpurun_out/r4f; mkdir -p $O
cd $GRAFT_REPO_ROOT
run() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > $O/$n.log 2>&1; local rc=$?; echo "== $n rc=$rc"; tail -4 $O/$n.log | cut -c1-300; case $rc in 0) ;; *) exit $rc;; esac; }
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so MYFYP_F32_VARIANT=2 run stamps_v2 200 python scripts/probes/stamps_f32v2.py
MYFYP_F32_VARIANT=2 run bench_v2 200 python bench.py --steps 200 --warmup 10
MYFYP_F32_VARIANT=1 run bench_v1 200 python bench.py --steps 200 --warmup 10
