#!/bin/bash
# GPU validation: numerics tests, bench N=1 (graph + eager A/B), kernel-trace profile.
# Every GPU step has its own time limit; a crash/timeout/abort stops the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
stop_if_fatal() { case "$1" in 124|134|137|139) echo "fatal rc=$1 in $2"; exit "$1";; esac; }
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; tail -3 gpurun_out/gpu_tests.log; stop_if_fatal $rc pytest
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench1.log; exit 1; }
tail -1 gpurun_out/bench1.log; grep '^\[bench\]' gpurun_out/bench1.log | tail -5
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --eager > gpurun_out/bench1_eager.log 2>&1 || { echo "eager bench failed"; exit 1; }
tail -1 gpurun_out/bench1_eager.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*stats*"
