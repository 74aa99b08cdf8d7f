#!/bin/bash
# BASELINE configs 3-5 on the CNN engine.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-cnn}
mkdir -p $O
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
run() {
  local name=$1; shift
  timeout -k 10 400 python benchmarks/bench_cnn.py "$@" > $O/$name.log 2>&1
  rc=$?; stop_if_fatal $rc $name; [ $rc -ne 0 ] && { echo "$name failed"; tail -25 $O/$name.log; exit $rc; }
  echo "$name: $(grep '"value"' $O/$name.log | cut -c1-330)"
}
run lenet_ring --model lenet5 --aggregator neighbor --rounds 4
run resnet_fedavg --model resnet18 --rounds 3
run resnet_fedprox_drop --model resnet18 --aggregator fedprox --dirichlet 0.5 --dropout --rounds 3
