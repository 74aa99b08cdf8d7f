#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/cnn7; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -m pytest tests -x -q -m gpu -k cnn > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/gpu_tests.log; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/gpu_tests.log | head -30; exit $rc; }
timeout -k 10 300 python scripts/probes/conv_ab.py > $O/conv_shapes.log 2>&1 || { echo "probe failed"; tail -20 $O/conv_shapes.log; exit 1; }
grep -v amdgpu.ids $O/conv_shapes.log
timeout -k 10 600 python benchmarks/bench_cnn.py --model resnet18 --rounds 2 > $O/resnet.log 2>&1 || { echo "bench failed"; tail -30 $O/resnet.log; exit 1; }
grep -v amdgpu.ids $O/resnet.log | tail -1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 benchmarks/bench_cnn.py --model resnet18 --rounds 1 --n-train 8192 --n-test 1024 > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
