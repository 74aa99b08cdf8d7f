#!/bin/bash
# CNN engine after the Wf-layout gradient / fused optimizer change: GPU tests, config 3/4 benches, ResNet kernel profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/cnn4; mkdir -p $O
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -30; exit $rc; }
run() { local name=$1; shift; timeout -k 10 600 python benchmarks/bench_cnn.py "$@" > $O/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids $O/$name.log | tail -2; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; tail -30 $O/$name.log; exit $rc; }; }
run cnn_resnet_fedavg --model resnet18 --rounds 2
run cnn_lenet_ring --model lenet5 --aggregator neighbor --rounds 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_cnn -o run -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --n-train 8192 --n-test 1024 > $O/prof_cnn.log 2>&1 || { echo "prof failed"; tail -20 $O/prof_cnn.log; exit 1; }
head -14 $O/prof_cnn/run_kernel_stats.csv | cut -c1-120
