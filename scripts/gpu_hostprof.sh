#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-hostprof}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 3 > $O/bench_$i.log 2>&1
  rc=$?; stop_if_fatal $rc bench$i; tail -1 $O/bench_$i.log | cut -c90-150
done
timeout -k 10 300 python scripts/probes/py_profile_bench.py --steps 30 --warmup 3 > $O/pyprof.log 2>&1
rc=$?; stop_if_fatal $rc pyprof
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/p -o run -- python3 bench.py --steps 20 --warmup 2 > $O/p.log 2>&1
rc=$?; stop_if_fatal $rc trace; tail -1 $O/p.log | cut -c90-150
