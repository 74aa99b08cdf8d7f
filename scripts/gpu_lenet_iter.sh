#!/bin/bash
# Fused LeNet iteration: phase stamps, numerics tests, config-3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-leniter}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
MYFYP_NATIVE_LIB=build/stamps/libmyfyp_hip.so timeout -k 10 300 python scripts/probes/lenet_stamps.py > $O/stamps.log 2>&1
rc=$?; tail -15 $O/stamps.log; stop_if_fatal $rc stamps; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_cnn_engine_gpu.py -k "lenet or graph_replay" -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; stop_if_fatal $rc tests; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -30; exit $rc; }
timeout -k 10 300 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 4 > $O/lenet_ring.log 2>&1
rc=$?; stop_if_fatal $rc bench; [ $rc -ne 0 ] && { tail -20 $O/lenet_ring.log; exit $rc; }
grep '"value"' $O/lenet_ring.log | cut -c1-300; grep "median ms" $O/lenet_ring.log
