#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-bench3}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
for i in 1 2 3; do
  timeout -k 10 240 python bench.py > $O/bench_$i.log 2>&1
  rc=$?; stop_if_fatal $rc bench$i; [ $rc -ne 0 ] && { tail -20 $O/bench_$i.log; exit $rc; }
  grep "round-end" $O/bench_$i.log; tail -1 $O/bench_$i.log | cut -c90-240
done
