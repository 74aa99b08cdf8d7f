#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-pyprof}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 python scripts/probes/py_profile_bench.py --steps 30 --warmup 3 > $O/pyprof.log 2>&1
rc=$?; stop_if_fatal $rc pyprof; grep '"value"' $O/pyprof.log | cut -c1-160
MYFYP_MLP_PERSISTENT=0 timeout -k 10 240 python bench.py --steps 30 --warmup 3 > $O/bench_steps.log 2>&1
rc=$?; stop_if_fatal $rc steps; tail -1 $O/bench_steps.log | cut -c1-160
timeout -k 10 240 python bench.py --steps 30 --warmup 3 > $O/bench_p.log 2>&1
rc=$?; stop_if_fatal $rc p; tail -1 $O/bench_p.log | cut -c1-160
