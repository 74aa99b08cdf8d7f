#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 600 python benchmarks/bench_cnn.py "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -2; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; exit $rc; }; }
run cnn_lenet_ring --model lenet5 --aggregator neighbor --rounds 5 --torch-step
run cnn_resnet_fedprox_drop --model resnet18 --aggregator fedprox --dirichlet 0.5 --dropout --rounds 3
