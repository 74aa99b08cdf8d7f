#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-hiptrace}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/p -o run -- python3 bench.py --steps 10 --warmup 2 > $O/p.log 2>&1
rc=$?; stop_if_fatal $rc p; tail -1 $O/p.log | cut -c1-200
MYFYP_MLP_PERSISTENT=0 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $O/s -o run -- python3 bench.py --steps 10 --warmup 2 > $O/s.log 2>&1
rc=$?; stop_if_fatal $rc s; tail -1 $O/s.log | cut -c1-200
ls $O/p $O/s
