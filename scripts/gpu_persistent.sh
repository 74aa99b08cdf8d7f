#!/bin/bash
# Persistent MLP epoch kernel: numerics tests, then headline bench A/B (persistent vs 3-launch steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-persist}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log; stop_if_fatal $rc tests; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python bench.py --steps 30 --warmup 3 > $O/bench_persistent.log 2>&1
rc=$?; stop_if_fatal $rc bench_p; [ $rc -ne 0 ] && { tail -30 $O/bench_persistent.log; exit $rc; }
tail -2 $O/bench_persistent.log | cut -c1-400
MYFYP_MLP_PERSISTENT=0 timeout -k 10 240 python bench.py --steps 30 --warmup 3 > $O/bench_steps.log 2>&1
rc=$?; stop_if_fatal $rc bench_s
tail -1 $O/bench_steps.log | cut -c1-300
timeout -k 10 240 python bench.py --steps 30 --warmup 3 --peers 1 > $O/bench_persistent_peers1.log 2>&1
rc=$?; stop_if_fatal $rc bench_p1
tail -1 $O/bench_persistent_peers1.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1
rc=$?; stop_if_fatal $rc prof
find $O/prof -name "*kernel_stats*"
