#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-stamps2}
mkdir -p $O
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so OPT=sgd timeout -k 10 200 python scripts/probes/stamps_persistent.py > $O/stamps_sgd.log 2>&1
rc=$?; tail -9 $O/stamps_sgd.log | head -4; exit $rc
