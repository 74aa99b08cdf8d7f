#!/bin/bash
# MLP engine round restructuring check: persistent/collective GPU tests, bench x3, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-mlpround}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_collective_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; stop_if_fatal $rc tests; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" $O/tests.log | head -30; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 240 python bench.py > $O/bench_$i.log 2>&1
  rc=$?; stop_if_fatal $rc bench$i; [ $rc -ne 0 ] && { tail -20 $O/bench_$i.log; exit $rc; }
  tail -1 $O/bench_$i.log | cut -c90-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 2 > $O/prof.log 2>&1
rc=$?; stop_if_fatal $rc prof
