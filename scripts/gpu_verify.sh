#!/bin/bash
# Post-rebuild verification: GPU suite, smoke(), headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-verify}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; tail -3 $O/gpu_tests.log; stop_if_fatal $rc pytest
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; stop_if_fatal $rc smoke
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log
