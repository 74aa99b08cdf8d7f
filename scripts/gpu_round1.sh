#!/bin/bash
# GPU validation: numerics tests, bench N=1 (graph + eager A/B), kernel-trace profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench1.log; exit 1; }
tail -1 gpurun_out/bench1.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --eager > gpurun_out/bench1_eager.log 2>&1 || { echo "eager bench failed"; exit 1; }
tail -1 gpurun_out/bench1_eager.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*stats*" | head
