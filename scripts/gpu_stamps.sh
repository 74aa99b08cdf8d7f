#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-stamps}
mkdir -p $O
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so timeout -k 10 200 python scripts/probes/stamps_persistent.py > $O/stamps.log 2>&1
rc=$?; tail -12 $O/stamps.log; exit $rc
