#!/bin/bash
# Full GPU suite, smoke, three headline bench runs (variance), kernel stats profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-full}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; stop_if_fatal $rc pytest; [ $rc -ne 0 ] && { grep -E "FAIL|Error" $O/gpu_tests.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log | cut -c1-150; stop_if_fatal $rc smoke
for i in 1 2 3; do
  timeout -k 10 240 python bench.py > $O/bench_default_$i.log 2>&1
  rc=$?; stop_if_fatal $rc bench$i; tail -1 $O/bench_default_$i.log | cut -c90-200
done
timeout -k 10 240 python bench.py --steps 30 --warmup 3 --peers 1 > $O/bench_peers1.log 2>&1
rc=$?; stop_if_fatal $rc peers1; tail -1 $O/bench_peers1.log | cut -c90-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 2 > $O/prof.log 2>&1
rc=$?; stop_if_fatal $rc prof
