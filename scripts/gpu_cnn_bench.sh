#!/bin/bash
# CNN engine benches (configs 3-5) + kernel profile of the ResNet-18 round.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 600 python benchmarks/bench_cnn.py "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -2 gpurun_out/$name.log; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 gpurun_out/$name.log; exit $rc; }; }
run cnn_lenet_ring --model lenet5 --aggregator neighbor --rounds 3 --torch-step
run cnn_resnet_fedavg --model resnet18 --rounds 2 --torch-step
run cnn_resnet_fedprox_drop --model resnet18 --aggregator fedprox --dirichlet 0.5 --dropout --rounds 2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cnn -o run -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --n-train 8192 --n-test 1024 > gpurun_out/prof_cnn.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_cnn.log; exit 1; }
find gpurun_out/prof_cnn -name "*kernel_stats*"
