#!/bin/bash
# Kernel iteration loop: persistent-path numerics tests, phase stamps, headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-iter}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_collective_gpu.py -x -q -k "fused_mlp or persistent or collective" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; stop_if_fatal $rc tests; [ $rc -ne 0 ] && { grep -E "Error|assert" $O/tests.log | head; exit $rc; }
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so timeout -k 10 200 python scripts/probes/stamps_persistent.py > $O/stamps.log 2>&1
rc=$?; tail -16 $O/stamps.log; stop_if_fatal $rc stamps
timeout -k 10 240 python bench.py --steps 30 --warmup 3 > $O/bench.log 2>&1
rc=$?; stop_if_fatal $rc bench; tail -1 $O/bench.log | cut -c1-200
