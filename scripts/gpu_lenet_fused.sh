#!/bin/bash
# Fused LeNet-5 step: numerics vs torch / the layer-wise path, then config-3 bench + kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-lenetfused}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 400 python -u -m pytest tests/test_cnn_engine_gpu.py -k "lenet or graph_replay" -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; stop_if_fatal $rc tests; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -30; exit $rc; }
timeout -k 10 300 python benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 4 > $O/lenet_ring.log 2>&1
rc=$?; stop_if_fatal $rc bench; [ $rc -ne 0 ] && { tail -20 $O/lenet_ring.log; exit $rc; }
grep '"value"' $O/lenet_ring.log | cut -c1-420
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 2 > $O/lenet_prof.log 2>&1
rc=$?; stop_if_fatal $rc prof
head -8 $O/prof/run_kernel_stats.csv | cut -c1-160
