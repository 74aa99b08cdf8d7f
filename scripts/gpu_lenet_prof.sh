#!/bin/bash
# LeNet-5 (config 3) kernel-level profile + a roctx marker trace of the headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-lenetprof}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 benchmarks/bench_cnn.py --model lenet5 --aggregator neighbor --rounds 2 > $O/lenet_prof.log 2>&1
rc=$?; stop_if_fatal $rc lenet_prof; [ $rc -ne 0 ] && { tail -20 $O/lenet_prof.log; exit $rc; }
grep '"value"' $O/lenet_prof.log | cut -c1-200
MYFYP_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $O/markers -o run -- python3 bench.py --steps 5 --warmup 2 > $O/markers.log 2>&1
rc=$?; stop_if_fatal $rc markers; [ $rc -ne 0 ] && { tail -20 $O/markers.log; exit $rc; }
tail -1 $O/markers.log | cut -c1-160
ls -R $O/markers | head
